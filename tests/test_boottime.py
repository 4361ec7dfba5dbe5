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


def test_parse_time_offsets():
    # helm status -o json: Go RFC3339Nano with the client's local offset
    assert parse_k8s_time("2021-10-14T15:42:34.25+02:00") == 1634218954.25
    assert parse_k8s_time("2021-10-14T13:42:34.123456789Z") == pytest.approx(1634218954.123457)


def test_collect_cli_offline_fixtures(tmp_path, capsys):
    """helm status + DV/VMI JSON + guest stamps (as written by the chart's
    cloud-init, kvedge-ready.service and the module) -> boot_to_ready_s per replica and
    for the fleet.  Fixture inputs are labelled unmeasured."""
    from kvedge_amd.utils import boottime

    t0 = 1_700_000_000.0
    (tmp_path / "helm.json").write_text(json.dumps(
        {"info": {"first_deployed": "2023-11-14T22:13:20.000000000Z", "status": "deployed"}}))
    dv = {"status": {"phase": "Succeeded", "conditions": [
        {"type": "Ready", "status": "True", "lastTransitionTime": "2023-11-14T22:13:50Z"}]}}
    vmi = {"status": {"phaseTransitionTimestamps": [
        {"phase": "Running", "phaseTransitionTimestamp": "2023-11-14T22:13:58Z"}]}}
    args = ["collect", "--release", "rel", "--replicas", "2",
            "--helm-status-json", str(tmp_path / "helm.json")]
    for i, extra in enumerate((0.0, 7.0)):
        (tmp_path / f"dv{i}.json").write_text(json.dumps(dv))
        (tmp_path / f"vmi{i}.json").write_text(json.dumps(vmi))
        (tmp_path / f"st{i}").write_text(
            f"bootcmd {t0 + 50}\nconfig_applied {t0 + 61}\ngpu_ready {t0 + 62}\n"
            f"runcmd_done {t0 + 63}\nedge_agent_running {t0 + 70 + extra}\n"
            f"module_first_inference {t0 + 80 + extra}\niotedge_check_pass {t0 + 90 + extra}\n")
        args += ["--dv-json", str(tmp_path / f"dv{i}.json"), "--vmi-json",
                 str(tmp_path / f"vmi{i}.json"), "--stamps", str(tmp_path / f"st{i}")]
    assert boottime.main(args + ["--out", str(tmp_path / "out.json")]) == 0
    res = json.loads((tmp_path / "out.json").read_text())
    r0, r1 = res["replicas"]
    assert r0["vm"] == "aziot-edge-kubevirt-linux" and r1["vm"] == "aziot-edge-kubevirt-linux-1"
    assert r0["datavolume_succeeded_s"] == 30 and r0["vmi_running_s"] == 38
    assert r0["iotedge_check_pass_s"] == 90 and r0["boot_to_ready_s"] == 90
    assert r1["edge_agent_running_s"] == 77 and r1["module_first_inference_s"] == 87
    assert res["boot_to_ready_s"] == 97 and res["helm_to_edge_agent_s"] == 77
    assert res["measured"] is False and "unmeasured" in res["note"]
    assert res["reference"]["helm_to_edge_agent_s"] == [156.0, 216.0]


def test_collect_live_dry_run_commands():
    from kvedge_amd.utils import boottime

    import io
    import contextlib

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        boottime.main(["collect", "--release", "rel", "--replicas", "2", "--live", "--dry-run",
                       "--namespace", "edge", "--helm-install-epoch", "0"])
    res = json.loads(buf.getvalue())
    cmds = res["commands"]
    assert cmds[0] == "helm status rel -n edge -o json"
    assert "kubectl get datavolume aziot-edge-kubevirt-linux-dv-1 -n edge -o json" in cmds
    assert "kubectl get vmi aziot-edge-kubevirt-linux -n edge -o json" in cmds
    assert any(c.startswith("virtctl ssh -n edge") and "ubuntu@vmi/aziot-edge-kubevirt-linux-1" in c
               for c in cmds)
    assert res["measured"] is False
