"""asciicast v2 reader + extraction of the reference demo's deployment timeline.

The reference (levi106/kvedge) publishes no benchmark numbers; its only measured
evidence is the real-time asciinema recording deployment/az-iot-edge-k8s-kubevirt-ascii.cast
(BASELINE.md).  This module parses such a recording and recovers the
boot-to-ready timeline (helm install -> DataVolume Succeeded -> VMI Running -> SSH ->
edgeAgent up) so the baseline numbers are reproducible from the file itself
(tests/test_boottime.py).  Works on any cast of the same runbook (e.g. a kvedge run).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

_ANSI = re.compile(r"\x1b\[[0-9;?]*[A-Za-z]|\x1b\][^\x07]*\x07")


@dataclass
class Cast:
    header: Dict
    events: List[Tuple[float, str, str]]  # (t, kind, data)

    @property
    def start_epoch(self) -> float:
        return float(self.header.get("timestamp", 0))

    def outputs(self):
        for i, (t, k, d) in enumerate(self.events):
            if k == "o":
                yield i, t, _ANSI.sub("", d)

    def find(self, pattern: str, after: float = -1.0) -> Optional[Tuple[int, float, re.Match]]:
        rx = re.compile(pattern)
        for i, t, d in self.outputs():
            if t <= after:
                continue
            m = rx.search(d)
            if m:
                return i, t, m
        return None

    def find_all(self, pattern: str):
        rx = re.compile(pattern)
        for i, t, d in self.outputs():
            for m in rx.finditer(d):
                yield i, t, m


def load(path: str) -> Cast:
    with open(path, encoding="utf-8") as f:
        header = json.loads(f.readline())
        if header.get("version") != 2:
            raise ValueError("only asciicast v2 is supported")
        events = []
        for ln in f:
            ln = ln.strip()
            if ln:
                t, k, d = json.loads(ln)
                events.append((float(t), k, d))
    return Cast(header, events)


def parse_age(s: str) -> float:
    """kubectl AGE ('90s', '2m51s', '3m12s', '1h2m') -> seconds."""
    tot = 0.0
    for n, u in re.findall(r"(\d+)([dhms])", s):
        tot += int(n) * {"d": 86400, "h": 3600, "m": 60, "s": 1}[u]
    return tot


def parse_up(s: str) -> Tuple[float, float]:
    """docker/iotedge 'Up 2 minutes' / 'Up a minute' -> (lo, hi) seconds bracket."""
    s = s.strip()
    m = re.match(r"Up (?:(about )?an? (minute|hour)|(\d+) (seconds|minutes|hours)|less than a second)", s)
    if not m:
        raise ValueError(s)
    if m.group(2):
        unit = 60 if m.group(2) == "minute" else 3600
        return float(unit), float(2 * unit)
    if m.group(3):
        n = int(m.group(3))
        unit = {"seconds": 1, "minutes": 60, "hours": 3600}[m.group(4)]
        return float(n * unit), float((n + 1) * unit)
    return 0.0, 1.0


@dataclass
class DeployTimeline:
    helm_submit_t: Optional[float] = None
    helm_deployed_t: Optional[float] = None
    release_epoch: Optional[int] = None
    dv_samples: List[Tuple[float, str, str, float]] = field(default_factory=list)  # t, phase, prog, age
    dv_succeeded_age_s: Optional[float] = None
    vmi_running_t: Optional[float] = None
    vmi_running_age_s: Optional[float] = None
    ssh_login_t: Optional[float] = None
    edge_agent_t: Optional[float] = None
    edge_agent_up_s: Optional[Tuple[float, float]] = None
    modules_seen: Dict[str, float] = field(default_factory=dict)
    cast_epoch: float = 0.0

    def metrics(self) -> Dict[str, object]:
        """BASELINE.md rows, seconds relative to `helm install` deployed."""
        out: Dict[str, object] = {}
        t0 = self.helm_deployed_t
        if self.release_epoch is not None and self.cast_epoch:
            t0 = self.release_epoch - self.cast_epoch  # release name = install epoch
        if self.helm_submit_t is not None and self.helm_deployed_t is not None:
            out["helm_install_cli_s"] = round(self.helm_deployed_t - self.helm_submit_t, 2)
        if self.dv_succeeded_age_s is not None:
            out["datavolume_import_le_s"] = self.dv_succeeded_age_s
            lower = [a for _, ph, _, a in self.dv_samples if ph != "Succeeded"]
            if lower:
                out["datavolume_import_gt_s"] = max(lower)
        if self.vmi_running_age_s is not None:
            out["helm_to_vmi_running_le_s"] = self.vmi_running_age_s
        if self.ssh_login_t is not None and t0 is not None:
            out["helm_to_ssh_le_s"] = round(self.ssh_login_t - t0, 1)
        if self.edge_agent_t is not None and t0 is not None and self.edge_agent_up_s:
            lo, hi = self.edge_agent_up_s
            seen = self.edge_agent_t - t0
            out["helm_to_edgeagent_s"] = (round(seen - hi, 1), round(seen - lo, 1))
            out["helm_to_edgeagent_observed_le_s"] = round(seen, 1)
        return out


def deployment_timeline(cast: Cast) -> DeployTimeline:
    tl = DeployTimeline(cast_epoch=cast.start_epoch)
    dep = cast.find(r"(?s)NAME: (\S+?)-(\d{10})\s.*?LAST DEPLOYED") or cast.find(r"LAST DEPLOYED")
    if dep:
        i, t, m = dep
        tl.helm_deployed_t = t
        if m.lastindex and m.lastindex >= 2:
            tl.release_epoch = int(m.group(2))
        # end of the echoed `helm install ... --set-file azIotEdgeConfig=...` command line
        # (BASELINE.md's "helm install CLI -> release deployed" start point)
        for j in range(i - 1, max(-1, i - 400), -1):
            tj, k, d = cast.events[j]
            if k == "o" and "EdgeConfig=" in d:
                tl.helm_submit_t = tj
                break
    for _, t, m in cast.find_all(r"(\S+-linux-dv)\s+(\w+)\s+([\d.]+%|N/A)?\s*(\d*)\s+((?:\d+[dhms])+)"):
        phase, prog, age = m.group(2), m.group(3) or "", parse_age(m.group(5))
        tl.dv_samples.append((t, phase, prog, age))
        if phase == "Succeeded" and tl.dv_succeeded_age_s is None:
            tl.dv_succeeded_age_s = age
    for _, t, m in cast.find_all(r"(\S+-linux)\s+((?:\d+[dhms])+)\s+Running\s"):
        if tl.vmi_running_t is None:
            tl.vmi_running_t, tl.vmi_running_age_s = t, parse_age(m.group(2))
    w = cast.find(r"Welcome to Ubuntu")
    if w:
        tl.ssh_login_t = w[1]
    ea = cast.find(r"edgeAgent\s+running\s+(Up [^\r\n]*?)\s{2,}")
    if ea:
        tl.edge_agent_t = ea[1]
        tl.edge_agent_up_s = parse_up(ea[2].group(1))
    for _, t, m in cast.find_all(r"\n(\w+)\s+running\s+Up "):
        tl.modules_seen.setdefault(m.group(1), t)
    return tl
