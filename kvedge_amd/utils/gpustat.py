"""GPU utilisation / HBM fields for module telemetry.

Sources, cheapest first, each optional:
  * torch.cuda.mem_get_info -> HBM used/total of this process's device (always there on
    a GPU; no subprocess);
  * ``amd-smi metric -g <i> -u -m --json`` -> GFX activity % (and VRAM as a cross-check).
    Called at telemetry cadence only, with a short timeout; if the tool is missing or
    fails once it is not tried again (``GpuStat.smi_ok``).
Fields that cannot be read are simply absent -- telemetry never fails because of them.
"""
from __future__ import annotations

import json
import shutil
import subprocess
from typing import Any, Dict, Optional


def _find(obj: Any, key: str):
    """First value under ``key`` anywhere in a nested JSON structure."""
    if isinstance(obj, dict):
        if key in obj:
            return obj[key]
        for v in obj.values():
            r = _find(v, key)
            if r is not None:
                return r
    elif isinstance(obj, list):
        for v in obj:
            r = _find(v, key)
            if r is not None:
                return r
    return None


def _num(v) -> Optional[float]:
    """amd-smi values come as numbers, "12 %" strings or {"value": 12, "unit": "%"}."""
    if isinstance(v, dict):
        v = v.get("value")
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, str):
        tok = v.strip().split()
        try:
            return float(tok[0]) if tok else None
        except ValueError:
            return None
    return None


def parse_amd_smi_metric(text: str) -> Dict[str, float]:
    """`amd-smi metric -u -m --json` output -> {util_pct, vram_used_mb, vram_total_mb}."""
    try:
        data = json.loads(text)
    except ValueError:
        return {}
    out = {}
    for k_out, k_in in (("util_pct", "gfx_activity"), ("vram_used_mb", "used_vram"),
                        ("vram_total_mb", "total_vram")):
        v = _num(_find(data, k_in))
        if v is not None:
            out[k_out] = v
    return out


class GpuStat:
    def __init__(self, device_index: int = 0, use_smi: bool = True, timeout_s: float = 2.0):
        self.index = device_index
        self.timeout_s = timeout_s
        self.smi = shutil.which("amd-smi") if use_smi else None
        self.smi_ok = self.smi is not None

    def sample(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        try:
            import torch

            if torch.cuda.is_available():
                free, total = torch.cuda.mem_get_info(self.index)
                out["hbm_used_gb"] = round((total - free) / 2 ** 30, 2)
                out["hbm_total_gb"] = round(total / 2 ** 30, 2)
        except Exception:  # noqa: BLE001 -- observability must never break serving
            pass
        if self.smi_ok:
            try:
                r = subprocess.run([self.smi, "metric", "-g", str(self.index), "-u", "-m",
                                    "--json"], capture_output=True, text=True,
                                   timeout=self.timeout_s)
                m = parse_amd_smi_metric(r.stdout) if r.returncode == 0 else {}
                if not m:
                    self.smi_ok = False
                if "util_pct" in m:
                    out["util_pct"] = m["util_pct"]
            except (OSError, subprocess.TimeoutExpired):
                self.smi_ok = False
        return out
