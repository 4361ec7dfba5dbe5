"""GPU utilisation / HBM fields for module telemetry.

Sources, cheapest first, each optional:
  * torch.cuda.mem_get_info -> HBM used/total of this process's device (always there on
    a GPU; no subprocess);
  * ``amd-smi metric -g <i> -u -m --json`` -> GFX activity % (and VRAM as a cross-check).
    Called at telemetry cadence only (rank 0 only in a fleet), with a short timeout; if
    the tool is missing or fails once it is not tried again (``GpuStat.smi_ok``).
    ``<i>`` is amd-smi's own enumeration index, found ONCE by PCI bus id
    (``amd-smi list --json``), never the HIP ordinal: HIP_/ROCR_VISIBLE_DEVICES renumber
    HIP devices but not amd-smi's.
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


def _norm_bdf(bdf: str) -> str:
    """'0000:05:00.0' / '05:00.0' / '0x5' bus forms -> 'DDDD:BB:DD.F' lower case."""
    b = bdf.strip().lower()
    if b.count(":") == 1:
        b = "0000:" + b
    return b


def smi_index_for_bdf(list_json: str, bdf: str) -> Optional[int]:
    """amd-smi's GPU index for a PCI address, from ``amd-smi list --json``
    ([{"gpu": 0, "bdf": "0000:05:00.0", ...}, ...])."""
    try:
        data = json.loads(list_json)
    except ValueError:
        return None
    want = _norm_bdf(bdf)
    for ent in data if isinstance(data, list) else data.get("gpu_list", []):
        if isinstance(ent, dict) and _norm_bdf(str(ent.get("bdf", ""))) == want:
            try:
                return int(ent.get("gpu"))
            except (TypeError, ValueError):
                return None
    return None


def torch_device_bdf(device_index: int) -> Optional[str]:
    """PCI address of a HIP device as torch reports it (None if unknown)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:  # noqa: BLE001
        return None


class GpuStat:
    def __init__(self, device_index: int = 0, use_smi: bool = True, timeout_s: float = 2.0):
        self.index = device_index  # HIP ordinal (torch.cuda)
        self.timeout_s = timeout_s
        self.smi = shutil.which("amd-smi") if use_smi else None
        self.smi_ok = self.smi is not None
        self.smi_index: Optional[int] = None  # amd-smi's index, resolved on first sample

    def _resolve_smi_index(self) -> Optional[int]:
        bdf = torch_device_bdf(self.index)
        if bdf is None:
            return None
        r = subprocess.run([self.smi, "list", "--json"], capture_output=True, text=True,
                           timeout=self.timeout_s)
        return smi_index_for_bdf(r.stdout, bdf) if r.returncode == 0 else None

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
                if self.smi_index is None:
                    self.smi_index = self._resolve_smi_index()
                    if self.smi_index is None:  # cannot map the device: do not guess
                        self.smi_ok = False
                        return out
                r = subprocess.run([self.smi, "metric", "-g", str(self.smi_index), "-u", "-m",
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
