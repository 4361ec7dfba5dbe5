"""N21: boot-timing tooling.  The reference's own recording is the fixture for the
baseline numbers; kvedge's timeline is computed from k8s JSON + stamps."""
import json
import os

import pytest

from kvedge_amd.utils import asciicast
from kvedge_amd.utils.boottime import BootTimeline, parse_k8s_time, parse_stamps

CAST = "/root/reference/deployment/az-iot-edge-k8s-kubevirt-ascii.cast"


@pytest.mark.skipif(not os.path.exists(CAST), reason="reference recording not mounted")
def test_reference_cast_reproduces_baseline_md():
    tl = asciicast.deployment_timeline(asciicast.load(CAST))
    m = tl.metrics()
    assert tl.release_epoch == 1634218954
    assert m["helm_install_cli_s"] == pytest.approx(5.5, abs=0.1)        # BASELINE row 1
    assert m["datavolume_import_gt_s"] == 90 and m["datavolume_import_le_s"] == 171
    assert m["helm_to_vmi_running_le_s"] == 192
    assert m["helm_to_ssh_le_s"] == pytest.approx(287, abs=1)
    lo, hi = m["helm_to_edgeagent_s"]                                     # boot-to-ready
    assert lo == pytest.approx(156, abs=1) and hi == pytest.approx(216, abs=1)
    assert m["helm_to_edgeagent_observed_le_s"] == pytest.approx(336, abs=1)
    assert "SimulatedTemperatureSensor" in tl.modules_seen


def test_parse_helpers():
    assert asciicast.parse_age("2m51s") == 171 and asciicast.parse_age("90s") == 90
    assert asciicast.parse_up("Up 2 minutes") == (120, 180)
    assert asciicast.parse_up("Up a minute") == (60, 120)
    assert parse_k8s_time("2021-10-14T13:42:34Z") == 1634218954
    assert parse_k8s_time("2021-10-14T13:42:34.5Z") == 1634218954.5


def test_boot_timeline_from_k8s_and_guest():
    t0 = 1_700_000_000.0
    dv = {"status": {"phase": "Succeeded", "conditions": [
        {"type": "Bound", "status": "True", "lastTransitionTime": "2023-11-14T22:13:25Z"},
        {"type": "Ready", "status": "True", "lastTransitionTime": "2023-11-14T22:13:50Z"}]}}
    vmi = {"status": {"phaseTransitionTimestamps": [
        {"phase": "Scheduling", "phaseTransitionTimestamp": "2023-11-14T22:13:51Z"},
        {"phase": "Running", "phaseTransitionTimestamp": "2023-11-14T22:13:58Z"}]}}
    stamps = f"bootcmd {t0 + 70}\nconfig_applied {t0 + 81}\ngpu_ready {t0 + 84}\nruncmd_done {t0 + 85}\n" \
             f"bootcmd {t0 + 500}\n"
    tl = BootTimeline.from_files(t0, json.dumps(dv), json.dumps(vmi), stamps, module_first=t0 + 95,
                                 check_pass=t0 + 99)
    s = tl.summary()
    assert s["datavolume_succeeded_s"] == 30 and s["vmi_running_s"] == 38
    assert s["guest_gpu_ready_s"] == 84 and s["boot_to_ready_s"] == 99
    assert "bootcmd#2" in parse_stamps(stamps)
