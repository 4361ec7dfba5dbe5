"""T-chart / T-cloudinit: offline rendering of the Helm chart.

Resource names must equal the reference's for replica 0;
new knobs (replicas, GPU passthrough, storage, eviction) render as designed; the
cloud-init scripts are executed against a fake root.
"""
import base64
import json
import os
import subprocess

import pytest
import yaml

from kvedge_amd.deploy.gotemplate import Renderer, TemplateError
from kvedge_amd.deploy.helm import Chart, apply_sets, manifests

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHART = os.path.join(ROOT, "deploy", "helm")
REF_CHART = "/root/reference/deployment/helm"
A1 = {  # SURVEY.md Appendix A.1, nameOverride=aziot-edge-kubevirt
    ("Secret", "aziot-edge-kubevirt-vm-aziotedgeconfig"),
    ("Secret", "aziot-edge-kubevirt-vm-cloudconfig"),
    ("DataVolume", "aziot-edge-kubevirt-linux-dv"),
    ("VirtualMachine", "aziot-edge-kubevirt-linux"),
    ("Service", "aziot-edge-kubevirt-vm-ssh-service"),
}
CFG = '[provisioning]\nsource = "manual"\nconnection_string = "HostName=x;DeviceId=y;SharedAccessKey=z"\n'


def render(sets=(), set_strings=(), files=(), name="rel"):
    ch = Chart(CHART)
    out = ch.render(name, sets=list(sets), set_strings=list(set_strings), set_files=list(files))
    return out, manifests(out)


def by_kind(objs, kind):
    return [o for o in objs if o["kind"] == kind]


@pytest.fixture
def cfg_file(tmp_path):
    p = tmp_path / "config.toml"
    p.write_text(CFG)
    return str(p)


@pytest.mark.skipif(not os.path.isdir(REF_CHART), reason="reference chart not mounted")
def test_renderer_on_reference_chart_matches_appendix_a1():
    ch = Chart(REF_CHART)
    out = ch.render("chart-1634218954", sets=["publicSshKey=k,aziotEdgeVmEnableExternalSsh=true"],
                    set_strings=["azIotEdgeConfig=" + CFG])
    objs = manifests(out)
    assert {(o["kind"], o["metadata"]["name"]) for o in objs} == A1
    # reference quirk A.2#7: a STRING "true" disables the reference's Service
    out2 = ch.render("r", set_strings=["aziotEdgeVmEnableExternalSsh=true"])
    assert not by_kind(manifests(out2), "Service")
    assert "kubectl get vmi aziot-edge-kubevirt-linux" in out["NOTES.txt"]


def test_default_render_keeps_reference_names(cfg_file):
    out, objs = render(sets=["publicSshKey=ssh-ed25519 AAAA"], files=["azIotEdgeConfig=" + cfg_file])
    names = {(o["kind"], o["metadata"]["name"]) for o in objs if o["kind"] != "ConfigMap"}
    assert names == A1
    vm = by_kind(objs, "VirtualMachine")[0]
    assert vm["apiVersion"] == "kubevirt.io/v1"
    assert vm["spec"]["runStrategy"] == "Always"
    labels = vm["spec"]["template"]["metadata"]["labels"]
    assert labels["kubevirt.io/domain"] == "aziot-edge-kubevirt-vm"
    assert labels["app.kubernetes.io/version"] == "0.2.0"
    assert labels["app.kubernetes.io/managed-by"] == "Helm"
    assert labels["helm.sh/chart"] == "aziot-edge-kubevirt-0.2.0"
    svc = by_kind(objs, "Service")[0]
    assert svc["spec"]["selector"]["kubevirt.io/domain"] == labels["kubevirt.io/domain"]
    assert svc["spec"]["type"] == "LoadBalancer" and svc["spec"]["ports"][0]["port"] == 22
    dv = by_kind(objs, "DataVolume")[0]
    assert dv["spec"]["pvc"]["resources"]["requests"]["storage"] == "40Gi"
    assert dv["spec"]["source"]["registry"]["url"].startswith("docker://")
    assert vm["spec"]["template"]["spec"]["volumes"][0]["dataVolume"]["name"] == dv["metadata"]["name"]
    iface = vm["spec"]["template"]["spec"]["domain"]["devices"]["interfaces"][0]
    assert iface["macAddress"] == "fe:7e:48:a0:7d:22" and "masquerade" in iface


def test_config_secret_roundtrip(cfg_file):
    _, objs = render(files=["azIotEdgeConfig=" + cfg_file])
    sec = [o for o in by_kind(objs, "Secret") if o["metadata"]["name"].endswith("aziotedgeconfig")][0]
    assert base64.b64decode(sec["data"]["userdata"]).decode() == CFG


def _cloudinit(objs, i=0):
    sec = [o for o in by_kind(objs, "Secret") if "cloudconfig" in o["metadata"]["name"]][i]
    txt = base64.b64decode(sec["data"]["userdata"]).decode()
    return txt, yaml.safe_load(txt)


def test_cloudinit_contract():
    _, objs = render(sets=["publicSshKey=ssh-ed25519 KEY"])
    txt, ci = _cloudinit(objs)
    assert txt.startswith("#cloud-config\n")
    assert ci["hostname"] == "iotedgevm" and ci["ssh_authorized_keys"] == ["ssh-ed25519 KEY"]
    vm = by_kind(objs, "VirtualMachine")[0]
    serial = [d for d in vm["spec"]["template"]["spec"]["domain"]["devices"]["disks"]
              if d["name"] == "aziotedgeconfigdisk"][0]["serial"]
    assert serial == "D23YZ9W6WA5DJ487"
    assert any(serial in " ".join(map(str, c)) for c in ci["bootcmd"])
    paths = {f["path"] for f in ci["write_files"]}
    assert "/usr/local/sbin/kvedge-apply-config" in paths
    assert "apt" not in ci  # pre-baked image: nothing to install at boot
    flat = [" ".join(map(str, c)) if isinstance(c, list) else c for c in ci["runcmd"]]
    assert any("enable --now kvedge-config.service" in c for c in flat)
    assert any("kvedge-gpu-check 1" in c for c in flat)
    # not pre-baked: jammy/noble Microsoft repo + installs, never bionic
    _, objs2 = render(sets=["image.prebaked=false"])
    txt2, ci2 = _cloudinit(objs2)
    assert "noble" in ci2["apt"]["sources"]["microsoft-prod.list"]["source"]
    assert "bionic" not in txt2
    assert any("aziot-edge" in " ".join(map(str, c)) for c in ci2["runcmd"])


def test_gpu_passthrough_and_firmware():
    _, objs = render(sets=["gpu.count=2"])
    spec = by_kind(objs, "VirtualMachine")[0]["spec"]["template"]
    hd = spec["spec"]["domain"]["devices"]["hostDevices"]
    assert [h["deviceName"] for h in hd] == ["amd.com/mi355x"] * 2
    assert spec["spec"]["domain"]["firmware"]["bootloader"]["efi"]["secureBoot"] is False
    ann = json.loads(spec["metadata"]["annotations"]["hooks.kubevirt.io/hookSidecars"])
    hook_cm = [o for o in by_kind(objs, "ConfigMap") if o["metadata"]["name"].endswith("mmio64-hook")][0]
    assert ann[0]["configMap"]["name"] == hook_cm["metadata"]["name"]
    assert "X-PciMmio64Mb,string=1048576" in hook_cm["data"]["hook.sh"]
    assert spec["spec"]["evictionStrategy"] == "None"  # VFIO: no live migration
    # CPU-only VM (BASELINE config 1): no host devices, no hook
    _, objs0 = render(sets=["gpu.count=0"])
    spec0 = by_kind(objs0, "VirtualMachine")[0]["spec"]["template"]
    assert "hostDevices" not in spec0["spec"]["domain"]["devices"]
    assert "annotations" not in spec0["metadata"]
    assert not [o for o in by_kind(objs0, "ConfigMap") if "mmio64" in o["metadata"]["name"]]


def test_replicas_scale_out(tmp_path):
    cfgs = []
    for i in range(3):
        p = tmp_path / f"c{i}.toml"
        p.write_text(f"device = {i}\n")
        cfgs.append(str(p))
    _, objs = render(sets=["replicas=3", "macAddresses[1]=fe:7e:48:a0:7d:23"],
                     files=[f"replicaConfigs[{i}]={c}" for i, c in enumerate(cfgs)])
    vms = by_kind(objs, "VirtualMachine")
    assert [v["metadata"]["name"] for v in vms] == [
        "aziot-edge-kubevirt-linux", "aziot-edge-kubevirt-linux-1", "aziot-edge-kubevirt-linux-2"]
    svcs = by_kind(objs, "Service")
    for vm, svc in zip(vms, svcs):
        assert svc["spec"]["selector"]["kubevirt.io/domain"] == \
            vm["spec"]["template"]["metadata"]["labels"]["kubevirt.io/domain"]
    secrets = [o for o in by_kind(objs, "Secret") if "aziotedgeconfig" in o["metadata"]["name"]]
    assert [base64.b64decode(s["data"]["userdata"]).decode() for s in secrets] == \
        [f"device = {i}\n" for i in range(3)]
    assert len(by_kind(objs, "DataVolume")) == 3
    macs = [v["spec"]["template"]["spec"]["domain"]["devices"]["interfaces"][0].get("macAddress")
            for v in vms]
    assert macs[1] == "fe:7e:48:a0:7d:23" and macs[2] is None
    hosts = [_cloudinit(objs, i)[1]["hostname"] for i in range(3)]
    assert hosts == ["iotedgevm", "iotedgevm-1", "iotedgevm-2"]


def test_ssh_flag_accepts_strings_and_bools():
    for v, want in (("true", 1), ("false", 0)):
        _, a = render(set_strings=[f"aziotEdgeVmEnableExternalSsh={v}"])
        _, b = render(sets=[f"aziotEdgeVmEnableExternalSsh={v}"])
        assert len(by_kind(a, "Service")) == want and len(by_kind(b, "Service")) == want


def test_names_truncation_and_empty_override():
    long = "a" * 39 + "-bbbbbbbb"
    _, objs = render(sets=[f"nameOverride={long}"])
    vm = by_kind(objs, "VirtualMachine")[0]
    assert vm["metadata"]["name"] == "a" * 39 + "-linux"
    _, objs = render(set_strings=["nameOverride="])
    names = {o["metadata"]["name"] for o in objs}
    assert "aziot-edge-kubevirt-vm-cloudconfig" in names  # fixed quirk A.2#2
    assert not any(n.startswith("-") for n in names)


def test_storage_and_http_source():
    _, objs = render(sets=["storage.accessMode=ReadWriteMany", "storage.className=ceph-rbd",
                           "image.source=http", "image.httpUrl=https://example/img.qcow2"])
    dv = by_kind(objs, "DataVolume")[0]["spec"]
    assert dv["pvc"]["accessModes"] == ["ReadWriteMany"]
    assert dv["pvc"]["storageClassName"] == "ceph-rbd"
    assert dv["source"]["http"]["url"] == "https://example/img.qcow2"
    with pytest.raises(TemplateError, match="httpUrl"):
        render(sets=["image.source=http"])


def test_module_deployment_manifest():
    _, objs = render(sets=["module.model=yolov8n", "module.batch=32"])
    cm = [o for o in by_kind(objs, "ConfigMap") if o["metadata"]["name"].endswith("module-deployment")][0]
    man = json.loads(cm["data"]["deployment.json"])["modulesContent"]
    mod = man["$edgeAgent"]["properties.desired"]["modules"]["kvedge"]
    co = json.loads(mod["settings"]["createOptions"])
    devs = {d["PathOnHost"] for d in co["HostConfig"]["Devices"]}
    assert devs == {"/dev/kfd", "/dev/dri"} and set(co["HostConfig"]["GroupAdd"]) == {"video", "render"}
    assert man["kvedge"]["properties.desired"]["model"] == "yolov8n"
    assert man["kvedge"]["properties.desired"]["batch"] == 32
    assert "FROM /messages/modules/kvedge/outputs/*" in \
        man["$edgeHub"]["properties.desired"]["routes"]["telemetryToCloud"]


def test_golden_default_render():
    out, _ = render(name="golden")
    got = "".join(f"---\n# {k}\n{v.strip()}\n" for k, v in sorted(out.items()))
    golden = os.path.join(CHART, "tests", "golden_default.yaml")
    if os.environ.get("KVEDGE_UPDATE_GOLDEN"):
        os.makedirs(os.path.dirname(golden), exist_ok=True)
        open(golden, "w").write(got)
    assert got == open(golden).read()


def test_set_parsing():
    v = apply_sets({"a": {"b": 1}}, sets=["a.c=true,x=3,s=str", "l[1]=z", r"k\.dot=1"],
                   set_strings=["n=007"])
    assert v == {"a": {"b": 1, "c": True}, "x": 3, "s": "str", "l": [None, "z"], "k.dot": 1,
                 "n": "007"}


def test_template_language_subset():
    r = Renderer()
    src = ('{{- define "t" -}}[{{ . }}]{{- end -}}'
           '{{ $x := 3 }}{{ range $i, $v := list "a" "b" }}{{ $i }}={{ $v }};{{ end }}'
           '{{ if and (gt $x 2) (not false) }}yes{{ else }}no{{ end }} '
           '{{ include "t" "q" | upper }} {{ printf "%s-%d" "n" 7 }} {{ "abc" | trunc 2 }} '
           '{{ with .m }}{{ .k }}{{ end }} {{ toJson (dict "b" 1 "a" (list 1 2)) }}')
    assert r.render(src, {"m": {"k": "K"}}) == '0=a;1=b;yes [Q] n-7 ab K {"a":[1,2],"b":1}'
    with pytest.raises(TemplateError):
        r.render("{{ eq 1 \"1\" }}", {})


def _fake_root_script(script: str, root) -> str:
    return (script.replace("/mnt/app-secret", f"{root}/mnt/app-secret")
            .replace("/etc/aziot", f"{root}/etc/aziot")
            .replace("/var/lib/kvedge", f"{root}/var/lib/kvedge")
            .replace("/usr/local/sbin/kvedge-stamp", f"{root}/stamp")
            .replace("/dev/kfd", f"{root}/dev/kfd").replace("/dev/dri", f"{root}/dev/dri"))


def test_cloudinit_scripts_in_fake_root(tmp_path):
    _, objs = render()
    _, ci = _cloudinit(objs)
    files = {f["path"]: f["content"] for f in ci["write_files"]}
    root = tmp_path
    for d in ("mnt/app-secret", "etc", "var/lib/kvedge", "bin", "dev/dri"):
        (root / d).mkdir(parents=True, exist_ok=True)
    (root / "stamp").write_text(_fake_root_script(files["/usr/local/sbin/kvedge-stamp"], root))
    (root / "stamp").chmod(0o755)
    log = root / "iotedge.log"
    (root / "bin" / "iotedge").write_text(f"#!/bin/sh\necho \"$@\" >> {log}\n")
    (root / "bin" / "iotedge").chmod(0o755)
    apply = root / "apply.sh"
    apply.write_text(_fake_root_script(files["/usr/local/sbin/kvedge-apply-config"], root))
    env = dict(os.environ, PATH=f"{root}/bin:" + os.environ["PATH"])
    run = lambda: subprocess.run(["sh", str(apply)], env=env, check=True, capture_output=True)  # noqa
    run()  # no config on the disk: nothing happens
    assert not log.exists()
    (root / "mnt/app-secret/userdata").write_text(CFG)
    run()
    assert (root / "etc/aziot/config.toml").read_text() == CFG
    assert log.read_text().count("config apply") == 1
    run()  # unchanged: idempotent, no re-apply
    assert log.read_text().count("config apply") == 1
    (root / "mnt/app-secret/userdata").write_text(CFG + "# rotated\n")
    run()
    assert log.read_text().count("config apply") == 2
    # GPU check: times out without devices, succeeds once /dev/kfd + a render node exist
    gpu = root / "gpu.sh"
    gpu.write_text(_fake_root_script(files["/usr/local/sbin/kvedge-gpu-check"], root))
    r = subprocess.run(["sh", str(gpu), "1", "1"], capture_output=True)
    assert r.returncode == 1
    (root / "dev/kfd").write_text("")
    (root / "dev/dri/renderD128").write_text("")
    r = subprocess.run(["sh", str(gpu), "1", "2"], capture_output=True)
    assert r.returncode == 0
    info = json.loads((root / "var/lib/kvedge/gpu.json").read_text())
    assert info["kfd"] is True and info["render_nodes"] == 1
    stamps = (root / "var/lib/kvedge/boot-timing").read_text()
    assert "config_applied" in stamps and "gpu_ready" in stamps
