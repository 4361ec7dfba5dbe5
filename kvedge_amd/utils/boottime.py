"""N21 boot-to-ready timing: `helm install` -> DataVolume Succeeded -> VMI Running ->
guest cloud-init stamps (config applied, GPU ready) -> edgeAgent running -> edge module
first inference -> `iotedge check` pass.

Producer: the chart's cloud-init (deploy/helm/templates/_helpers.tpl) stamps
bootcmd / config_applied / gpu_ready / runcmd_done, kvedge-ready.service stamps
edge_agent_running / iotedge_check_pass, and the module appends module_first_inference
-- all into the guest's /var/lib/kvedge/boot-timing.

Collector CLI (the reference measured the same chain by eye from its asciicast,
reference deployment/az-iot-edge-k8s-kubevirt-ascii.cast:2889-2890):

  python -m kvedge_amd.utils.boottime collect --release REL [--replicas N] \
      [--helm-status-json F | --helm-install-epoch E] [--dv-json F ...] [--vmi-json F ...] \
      [--stamps F ...]            # offline: files saved from a cluster
  python -m kvedge_amd.utils.boottime collect --release REL --live [--dry-run]
                                  # kubectl / helm / virtctl ssh against a cluster

Inputs are what a real run leaves behind, all optional:
  * `kubectl get datavolume <dv> -o json`  (status.conditions[].lastTransitionTime),
  * `kubectl get vmi <vm> -o json`         (status.phaseTransitionTimestamps[]),
  * the guest's /var/lib/kvedge/boot-timing stamp file (written by the chart's
    cloud-init: "<name> <epoch>" lines),
  * the module's first telemetry timestamp and an `iotedge check` pass epoch.
The reference measured the same chain by eye from its asciicast; the
asciicast path is :mod:`kvedge_amd.utils.asciicast`.
"""
from __future__ import annotations

import argparse
import calendar
import json
import re
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

# reference numbers (cast:2889-2890): helm install -> edgeAgent running
REFERENCE_BOOT_TO_READY_S = (156.0, 216.0)
REFERENCE_OBSERVED_READY_LE_S = 336.0
GUEST_STAMPS = ("bootcmd", "config_applied", "gpu_ready", "runcmd_done", "edge_agent_running",
                "module_first_inference", "iotedge_check_pass", "iotedge_check_timeout")


def parse_k8s_time(s: str) -> float:
    """RFC3339 '2021-10-14T13:45:25Z' / '...25.123456789+02:00' -> epoch seconds."""
    s = s.strip()
    off = 0
    m = re.search(r"([+-])(\d\d):(\d\d)$", s)
    if m and "T" in s[:m.start()]:
        off = (int(m.group(2)) * 3600 + int(m.group(3)) * 60) * (1 if m.group(1) == "+" else -1)
        s = s[:m.start()]
    s = s.rstrip("Z")
    frac = 0.0
    if "." in s:
        s, rest = s.split(".", 1)
        digits = "".join(ch for ch in rest if ch.isdigit())
        frac = float("0." + digits) if digits else 0.0
    return calendar.timegm(time.strptime(s, "%Y-%m-%dT%H:%M:%S")) + frac - off


def dv_succeeded_at(dv_json: dict) -> Optional[float]:
    st = dv_json.get("status", {})
    if st.get("phase") != "Succeeded":
        return None
    for c in st.get("conditions", []):
        if c.get("type") == "Ready" and c.get("status") == "True":
            return parse_k8s_time(c["lastTransitionTime"])
    return None


def vmi_running_at(vmi_json: dict) -> Optional[float]:
    for p in vmi_json.get("status", {}).get("phaseTransitionTimestamps", []):
        if p.get("phase") == "Running":
            return parse_k8s_time(p["phaseTransitionTimestamp"])
    return None


def parse_stamps(text: str) -> Dict[str, float]:
    """Guest stamp file -> {name: first epoch} (later duplicates = later boots, kept as name#n).
    Lines are ``<name> <epoch>`` or, since round 5, ``<name> <epoch> <boot id>``."""
    out: Dict[str, float] = {}
    for ln in text.splitlines():
        parts = ln.split()
        if len(parts) not in (2, 3):
            continue
        name, t = parts[0], float(parts[1])
        key, n = name, 1
        while key in out:
            n += 1
            key = f"{name}#{n}"
        out[key] = t
    return out


@dataclass
class BootTimeline:
    helm_install: float
    dv_succeeded: Optional[float] = None
    vmi_running: Optional[float] = None
    stamps: Dict[str, float] = field(default_factory=dict)
    module_first_inference: Optional[float] = None
    iotedge_check_pass: Optional[float] = None

    def summary(self) -> Dict[str, float]:
        t0 = self.helm_install
        out = {}

        def put(name, t):
            if t is not None:
                out[name] = round(t - t0, 3)

        put("datavolume_succeeded_s", self.dv_succeeded)
        put("vmi_running_s", self.vmi_running)
        for k in ("bootcmd", "config_applied", "gpu_ready", "runcmd_done"):
            put(f"guest_{k}_s", self.stamps.get(k))
        put("edge_agent_running_s", self.stamps.get("edge_agent_running"))
        put("module_first_inference_s",
            self.module_first_inference if self.module_first_inference is not None
            else self.stamps.get("module_first_inference"))
        put("iotedge_check_pass_s",
            self.iotedge_check_pass if self.iotedge_check_pass is not None
            else self.stamps.get("iotedge_check_pass"))
        # the headline: helm install -> `iotedge check` passes inside the guest
        if "iotedge_check_pass_s" in out:
            out["boot_to_ready_s"] = out["iotedge_check_pass_s"]
        if "iotedge_check_timeout" in self.stamps:
            out["iotedge_check_timed_out"] = True
        return out

    @staticmethod
    def from_files(helm_install_epoch: float, dv_json: Optional[str] = None,
                   vmi_json: Optional[str] = None, stamps: Optional[str] = None,
                   module_first: Optional[float] = None,
                   check_pass: Optional[float] = None) -> "BootTimeline":
        return BootTimeline(
            helm_install_epoch,
            dv_succeeded_at(json.loads(dv_json)) if dv_json else None,
            vmi_running_at(json.loads(vmi_json)) if vmi_json else None,
            parse_stamps(stamps) if stamps else {},
            module_first, check_pass)


# ---------------------------------------------------------------------------- collector
def helm_first_deployed(status_json: dict) -> float:
    """`helm status REL -o json` -> epoch of the install (info.first_deployed)."""
    return parse_k8s_time(status_json["info"]["first_deployed"])


class ClusterReader:
    """Reads the timeline inputs from a live cluster (kubectl, helm, virtctl ssh).
    ``dry_run`` records the command lines and returns nothing (no cluster in CI) -- the
    same adapter pattern as kvedge_amd.resilience.KubectlCluster."""

    def __init__(self, namespace: str = "default", dry_run: bool = False,
                 ssh_user: str = "ubuntu"):
        self.ns, self.dry_run, self.user = namespace, dry_run, ssh_user
        self.log: List[List[str]] = []

    def _run(self, *cmd: str) -> Optional[str]:
        self.log.append(list(cmd))
        if self.dry_run:
            return None
        r = subprocess.run(list(cmd), capture_output=True, text=True)
        return r.stdout if r.returncode == 0 else None

    def helm_status(self, release: str) -> Optional[str]:
        return self._run("helm", "status", release, "-n", self.ns, "-o", "json")

    def get_json(self, kind: str, name: str) -> Optional[str]:
        return self._run("kubectl", "get", kind, name, "-n", self.ns, "-o", "json")

    def guest_stamps(self, vmi: str) -> Optional[str]:
        return self._run("virtctl", "ssh", "-n", self.ns, "--local-ssh=false",
                         f"{self.user}@vmi/{vmi}", "--command",
                         "cat /var/lib/kvedge/boot-timing")


def collect(release: str, helm_install: Optional[float], dv_jsons: Sequence[Optional[str]],
            vmi_jsons: Sequence[Optional[str]], stamps: Sequence[Optional[str]],
            names: Sequence[str], measured: bool) -> dict:
    """Per-replica timelines + the fleet row set of BASELINE.md."""
    reps = []
    for i, name in enumerate(names):
        pick = lambda seq: seq[i] if i < len(seq) else None  # noqa: E731
        if helm_install is None:
            reps.append({"vm": name, "error": "no helm install epoch"})
            continue
        tl = BootTimeline.from_files(helm_install, pick(dv_jsons), pick(vmi_jsons), pick(stamps))
        reps.append(dict(vm=name, **tl.summary()))
    ready = [r["boot_to_ready_s"] for r in reps if "boot_to_ready_s" in r]
    agent = [r["edge_agent_running_s"] for r in reps if "edge_agent_running_s" in r]
    out = {"release": release, "helm_install_epoch": helm_install, "replicas": reps,
           "measured": measured,
           "reference": {"helm_to_edge_agent_s": list(REFERENCE_BOOT_TO_READY_S),
                         "helm_to_edge_agent_observed_le_s": REFERENCE_OBSERVED_READY_LE_S,
                         "iotedge_check_pass_s": None,
                         "source": "reference cast:2889-2890 (BASELINE.md)"}}
    if ready and len(ready) == len(names):
        out["boot_to_ready_s"] = max(ready)  # the fleet is ready when its last VM is
    if agent and len(agent) == len(names):
        out["helm_to_edge_agent_s"] = max(agent)
        out["vs_reference_edge_agent"] = round(REFERENCE_BOOT_TO_READY_S[0] / max(agent), 3)
    if not measured:
        out["note"] = "unmeasured: inputs are fixtures / dry-run, not a live cluster run"
    return out


def _read(path: Optional[str]) -> Optional[str]:
    if not path:
        return None
    with open(path) as f:
        return f.read()


def main(argv=None) -> int:
    from ..deploy.names import ChartNames

    ap = argparse.ArgumentParser(prog="python -m kvedge_amd.utils.boottime")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("collect", help="helm install -> iotedge check pass timeline")
    c.add_argument("--release", required=True)
    c.add_argument("--namespace", default="default")
    c.add_argument("--name-override", default="aziot-edge-kubevirt")
    c.add_argument("--replicas", type=int, default=1)
    c.add_argument("--helm-install-epoch", type=float, default=None)
    c.add_argument("--helm-status-json", default=None)
    c.add_argument("--dv-json", action="append", default=[])
    c.add_argument("--vmi-json", action="append", default=[])
    c.add_argument("--stamps", action="append", default=[])
    c.add_argument("--live", action="store_true", help="read everything from the cluster")
    c.add_argument("--dry-run", action="store_true", help="with --live: print the commands")
    c.add_argument("--measured", action="store_true",
                   help="the offline files were saved from a real cluster run")
    c.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    names = ChartNames(a.name_override, a.replicas)
    vms = [names.vm(i) for i in range(a.replicas)]
    if a.live:
        rd = ClusterReader(a.namespace, dry_run=a.dry_run)
        hs = rd.helm_status(a.release)
        t0 = helm_first_deployed(json.loads(hs)) if hs else a.helm_install_epoch
        dvs = [rd.get_json("datavolume", names.dv(i)) for i in range(a.replicas)]
        vmis = [rd.get_json("vmi", vm) for vm in vms]
        st = [rd.guest_stamps(vm) for vm in vms]
        res = collect(a.release, t0, dvs, vmis, st, vms, measured=not a.dry_run)
        if a.dry_run:
            res["commands"] = [" ".join(cmd) for cmd in rd.log]
    else:
        t0 = a.helm_install_epoch
        if a.helm_status_json:
            t0 = helm_first_deployed(json.loads(_read(a.helm_status_json)))
        res = collect(a.release, t0, [_read(p) for p in a.dv_json],
                      [_read(p) for p in a.vmi_json], [_read(p) for p in a.stamps], vms,
                      measured=a.measured)
    line = json.dumps(res, indent=1)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
