"""§5.5 observability: structured JSON logs and GPU telemetry fields (CPU tier)."""
import io
import json

from kvedge_amd.utils.gpustat import GpuStat, parse_amd_smi_metric
from kvedge_amd.utils.logging import get_logger, log_event


def test_json_log_lines():
    buf = io.StringIO()
    log = get_logger("kvedge.test_json", stream=buf)
    log_event(log, "rebuild", model="resnet50", batch=64, ok=True)
    rec = json.loads(buf.getvalue().strip())
    assert rec["event"] == "rebuild" and rec["level"] == "INFO"
    assert rec["model"] == "resnet50" and rec["batch"] == 64 and rec["ok"] is True
    assert rec["logger"] == "kvedge.test_json" and rec["ts"].endswith("Z")


def test_amd_smi_parser_variants():
    # value/unit objects (amd-smi >= 24.x) and "N %" strings both parse
    a = json.dumps([{"gpu": 0, "usage": {"gfx_activity": {"value": 87, "unit": "%"}},
                     "mem_usage": {"total_vram": {"value": 294896, "unit": "MB"},
                                   "used_vram": {"value": 51234, "unit": "MB"}}}])
    assert parse_amd_smi_metric(a) == {"util_pct": 87.0, "vram_used_mb": 51234.0,
                                       "vram_total_mb": 294896.0}
    b = json.dumps({"gpu_data": [{"usage": {"gfx_activity": "12 %"}}]})
    assert parse_amd_smi_metric(b) == {"util_pct": 12.0}
    assert parse_amd_smi_metric("not json") == {}


def test_gpustat_absent_tool_is_silent():
    s = GpuStat(0, use_smi=False)
    out = s.sample()  # CPU container: no GPU, no amd-smi -> empty, no exception
    assert isinstance(out, dict) and "util_pct" not in out


def test_amd_smi_parser_on_real_mi355x_output():
    """Fixture captured with `amd-smi metric -g 0 -u -m --json` on the MI355X pool."""
    import os

    p = os.path.join(os.path.dirname(__file__), "fixtures", "amdsmi_metric_mi355x.json")
    m = parse_amd_smi_metric(open(p).read())
    assert set(m) == {"util_pct", "vram_used_mb", "vram_total_mb"}
    assert m["vram_total_mb"] == 294896.0  # 288 GiB HBM3E


def test_amd_smi_index_is_mapped_by_pci_address():
    """amd-smi enumerates every GPU of the host; HIP ordinals follow
    HIP_/ROCR_VISIBLE_DEVICES.  The sampler maps by PCI bus id, never by ordinal."""
    from kvedge_amd.utils.gpustat import smi_index_for_bdf

    lst = json.dumps([{"gpu": 0, "bdf": "0000:05:00.0"}, {"gpu": 1, "bdf": "0000:15:00.0"},
                      {"gpu": 7, "bdf": "0000:F5:00.0"}])
    assert smi_index_for_bdf(lst, "0000:15:00.0") == 1
    assert smi_index_for_bdf(lst, "f5:00.0") == 7  # short form, case-insensitive
    assert smi_index_for_bdf(lst, "0000:25:00.0") is None
    assert smi_index_for_bdf("garbage", "0000:05:00.0") is None


def test_amd_smi_list_fixture_from_the_pool():
    """`amd-smi list --json` captured on the MI355X pool (r3 baseline run)."""
    import os

    from kvedge_amd.utils.gpustat import smi_index_for_bdf

    p = os.path.join(os.path.dirname(__file__), "fixtures", "amdsmi_list_mi355x.json")
    txt = open(p).read()
    bdf = json.loads(txt)[0]["bdf"]
    assert smi_index_for_bdf(txt, bdf) == 0
    assert smi_index_for_bdf(txt, bdf.upper()) == 0
