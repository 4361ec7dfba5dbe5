"""N21 boot-to-ready timing: `helm install` -> DataVolume Succeeded -> VMI Running ->
guest cloud-init stamps (config applied, GPU ready) -> edge module first inference ->
`iotedge check` pass.

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

import calendar
import json
import time
from dataclasses import dataclass, field
from typing import Dict, Optional


def parse_k8s_time(s: str) -> float:
    """RFC3339 '2021-10-14T13:45:25Z' (optionally with fraction) -> epoch seconds."""
    s = s.strip()
    frac = 0.0
    if "." in s:
        main, rest = s.split(".", 1)
        digits = "".join(ch for ch in rest if ch.isdigit())
        frac = float("0." + digits) if digits else 0.0
        s = main + "Z"
    return calendar.timegm(time.strptime(s.replace("Z", ""), "%Y-%m-%dT%H:%M:%S")) + frac


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
    """Guest stamp file -> {name: first epoch} (later duplicates = later boots, kept as name#n)."""
    out: Dict[str, float] = {}
    for ln in text.splitlines():
        parts = ln.split()
        if len(parts) != 2:
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
        put("module_first_inference_s", self.module_first_inference)
        put("iotedge_check_pass_s", self.iotedge_check_pass)
        ready = [v for k, v in out.items() if k in ("iotedge_check_pass_s",
                                                     "module_first_inference_s")]
        if ready:
            out["boot_to_ready_s"] = max(ready)
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
