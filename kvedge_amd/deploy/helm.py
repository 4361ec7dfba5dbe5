"""Offline `helm template` for the kvedge chart.

Loads a chart directory (Chart.yaml, values.yaml, templates/, .helmignore), merges
values the way Helm does (values files, then --set / --set-string / --set-file,
deep-merging maps), renders every non-partial template with
:mod:`kvedge_amd.deploy.gotemplate` and returns the manifests + NOTES.txt.

Reference behaviour reproduced: `helm install --generate-name . --set ...
--set-file azIotEdgeConfig=config.toml` (reference README.md:60) and the
.helmignore exclusion of files from packaging (reference .helmignore:24-25).
"""
from __future__ import annotations

import argparse
import copy
import fnmatch
import os
import re
import sys
import time
from typing import Dict, List, Optional, Tuple

import yaml

from .gotemplate import Renderer


def _load_helmignore(chart_dir: str) -> List[str]:
    p = os.path.join(chart_dir, ".helmignore")
    if not os.path.exists(p):
        return []
    pats = []
    for ln in open(p):
        ln = ln.strip()
        if ln and not ln.startswith("#"):
            pats.append(ln)
    return pats


def _ignored(rel: str, pats: List[str]) -> bool:
    base = os.path.basename(rel)
    for p in pats:
        p2 = p.rstrip("/")
        if fnmatch.fnmatch(rel, p2) or fnmatch.fnmatch(base, p2) or rel.startswith(p2 + "/"):
            return True
    return False


def deep_merge(base: dict, over: dict) -> dict:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = deep_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _typed(s: str):
    if s in ("true", "false"):
        return s == "true"
    if s == "null":
        return None
    if re.fullmatch(r"-?\d+", s):
        return int(s)
    return s


def _split_top(s: str) -> List[str]:
    """Split a --set string on commas not escaped with a backslash."""
    parts, cur, esc = [], [], False
    for c in s:
        if esc:
            cur.append(c if c == "," else "\\" + c)  # keep "\." for the key parser
            esc = False
        elif c == "\\":
            esc = True
        elif c == ",":
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(c)
    parts.append("".join(cur))
    return [p for p in parts if p]


def set_path(values: dict, path: str, value) -> None:
    keys = re.split(r"(?<!\\)\.", path)
    cur = values
    for k in keys[:-1]:
        k = k.replace("\\.", ".")
        m = re.fullmatch(r"(.+)\[(\d+)\]", k)
        if m:
            lst = cur.setdefault(m.group(1), [])
            idx = int(m.group(2))
            while len(lst) <= idx:
                lst.append({})
            cur = lst[idx]
        else:
            if not isinstance(cur.get(k), dict):
                cur[k] = {}
            cur = cur[k]
    last = keys[-1].replace("\\.", ".")
    m = re.fullmatch(r"(.+)\[(\d+)\]", last)
    if m:
        lst = cur.setdefault(m.group(1), [])
        idx = int(m.group(2))
        while len(lst) <= idx:
            lst.append(None)
        lst[idx] = value
    else:
        cur[last] = value


def apply_sets(values: dict, sets: List[str] = (), set_strings: List[str] = (),
               set_files: List[str] = ()) -> dict:
    v = copy.deepcopy(values)
    for s in sets or []:
        for kv in _split_top(s):
            k, _, val = kv.partition("=")
            set_path(v, k, _typed(val))
    for s in set_strings or []:
        for kv in _split_top(s):
            k, _, val = kv.partition("=")
            set_path(v, k, val)
    for s in set_files or []:
        k, _, fn = s.partition("=")
        with open(fn) as f:
            set_path(v, k, f.read())
    return v


class Chart:
    def __init__(self, chart_dir: str):
        self.dir = chart_dir
        with open(os.path.join(chart_dir, "Chart.yaml")) as f:
            self.meta = yaml.safe_load(f)
        vp = os.path.join(chart_dir, "values.yaml")
        self.values = yaml.safe_load(open(vp)) if os.path.exists(vp) else {}
        self.values = self.values or {}
        self.ignore = _load_helmignore(chart_dir)
        self.templates: Dict[str, str] = {}
        tdir = os.path.join(chart_dir, "templates")
        for root, _, files in os.walk(tdir):
            for fn in sorted(files):
                full = os.path.join(root, fn)
                rel = os.path.relpath(full, chart_dir)
                if _ignored(rel, self.ignore):
                    continue
                with open(full) as f:
                    self.templates[os.path.relpath(full, tdir)] = f.read()

    def chart_obj(self) -> dict:
        m = self.meta
        return {"Name": m.get("name"), "Version": str(m.get("version", "")),
                "AppVersion": str(m.get("appVersion", "")) if m.get("appVersion") else "",
                "Description": m.get("description", ""), "Type": m.get("type", "application"),
                "ApiVersion": m.get("apiVersion", "v2")}

    def render(self, release_name: Optional[str] = None, namespace: str = "default",
               values_files: List[str] = (), sets: List[str] = (), set_strings: List[str] = (),
               set_files: List[str] = (), is_upgrade: bool = False) -> Dict[str, str]:
        vals = copy.deepcopy(self.values)
        for vf in values_files or []:
            with open(vf) as f:
                vals = deep_merge(vals, yaml.safe_load(f) or {})
        vals = apply_sets(vals, sets, set_strings, set_files)
        name = release_name or f"{self.meta.get('name', 'chart')}-{int(time.time())}"
        ctx = {"Values": vals, "Chart": self.chart_obj(),
               "Release": {"Name": name, "Namespace": namespace, "Service": "Helm",
                           "IsInstall": not is_upgrade, "IsUpgrade": is_upgrade, "Revision": 1},
               "Capabilities": {"KubeVersion": {"Version": "v1.30.0", "Major": "1", "Minor": "30"},
                                "APIVersions": []},
               "Template": {"BasePath": "templates"}}
        r = Renderer()
        # partials first so every define is known
        for fn, src in sorted(self.templates.items()):
            if os.path.basename(fn).startswith("_"):
                r.add_source(src)
        out = {}
        for fn, src in sorted(self.templates.items()):
            if os.path.basename(fn).startswith("_"):
                continue
            ctx["Template"]["Name"] = f"{self.meta.get('name')}/templates/{fn}"
            out[fn] = r.render(src, ctx)
        return out


def manifests(rendered: Dict[str, str]) -> List[dict]:
    """Parse rendered templates (except NOTES.txt) into k8s objects."""
    objs = []
    for fn, txt in sorted(rendered.items()):
        if fn.endswith("NOTES.txt"):
            continue
        for doc in yaml.safe_load_all(txt):
            if doc:
                objs.append(doc)
    return objs


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m kvedge_amd.deploy.helm",
                                 description="offline helm template")
    ap.add_argument("cmd", choices=["template", "notes"])
    ap.add_argument("chart")
    ap.add_argument("--name", default=None)
    ap.add_argument("--namespace", default="default")
    ap.add_argument("-f", "--values", action="append", default=[])
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--set-string", action="append", default=[])
    ap.add_argument("--set-file", action="append", default=[])
    a = ap.parse_args(argv)
    ch = Chart(a.chart)
    out = ch.render(a.name, a.namespace, a.values, a.set, a.set_string, a.set_file)
    for fn, txt in sorted(out.items()):
        if fn.endswith("NOTES.txt"):
            if a.cmd == "notes":
                print(txt)
            continue
        if a.cmd == "template" and txt.strip():
            print(f"---\n# Source: {ch.meta.get('name')}/templates/{fn}")
            print(txt.strip("\n"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
