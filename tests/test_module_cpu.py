"""T-module: twin -> engine config, telemetry schema, direct methods,
checkpoint/resume, all through the fake edgeHub transport on CPU."""
import json

import pytest

from kvedge_amd.module.app import ModuleApp
from kvedge_amd.module.config import ModuleConfig
from kvedge_amd.module.transport import FakeTransport, StdoutTransport


class Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        self.t += 0.25
        return self.t


def test_config_patch_validation():
    c = ModuleConfig()
    c2 = c.apply_patch({"model": "yolov8n", "batch": "8", "$version": 3, "unknown": 1})
    assert c2.model == "yolov8n" and c2.batch == 8 and c2.needs_rebuild(c)
    assert not c2.apply_patch({"report_interval_s": 5}).needs_rebuild(c2)
    assert c2.resolved_image_size() == 640 and c.resolved_image_size() == 224
    for bad in ({"model": "vgg"}, {"batch": 0}, {"dtype": "fp32"}, {"image_size": 100},
                {"conf": 2}):
        with pytest.raises(ValueError):
            c.apply_patch(bad)


def test_simulated_temperature_module(tmp_path):
    tr = FakeTransport({"model": "simulated-temperature", "send_interval_s": 1.0,
                        "max_messages": 3})
    app = ModuleApp(tr, device="cpu", state_path=str(tmp_path / "s.json"), clock=Clock()).start()
    app.run(max_steps=40)
    msgs = tr.outputs("temperatureOutput")
    assert len(msgs) == 3  # capped like SimulatedTemperatureSensor's MessageCount
    assert {"machine", "ambient", "timeCreated"} <= set(msgs[0])
    assert tr.reported["config"]["model"] == "simulated-temperature"
    app.stop()


def test_heartbeat_outlives_the_message_cap_and_restarts(tmp_path):
    """the simulated sensor stops SENDING at max_messages, but the module
    is alive and its heartbeat must stay fresh -- also after a restart that resumes with
    the cap already reached (else `kvedge-health live` fails and KubeVirt restarts the VM
    forever).  The heartbeat runs on its own cadence (app.HEARTBEAT_S), not on sends."""
    from kvedge_amd.module import app as app_mod

    state, hb = str(tmp_path / "s.json"), tmp_path / "heartbeat"
    clk = Clock()
    cfg = {"model": "simulated-temperature", "send_interval_s": 1.0, "max_messages": 2,
           "report_interval_s": 600.0}
    tr = FakeTransport(cfg)
    a = ModuleApp(tr, device="cpu", state_path=state, clock=clk, heartbeat_path=str(hb)).start()
    a.run(max_steps=400)  # 100 s on the fake clock, far past the cap
    a.stop()
    assert len(tr.outputs("temperatureOutput")) == 2
    beats = []
    orig = ModuleApp._heartbeat

    def spy(self, msg):
        beats.append(self.clock.t)
        return orig(self, msg)

    ModuleApp._heartbeat = spy
    try:  # restart: the state file says the cap is reached; nothing is sent, beats go on
        tr2 = FakeTransport(cfg)
        clk2 = Clock()
        a2 = ModuleApp(tr2, device="cpu", state_path=state, clock=clk2,
                       heartbeat_path=str(hb)).start()
        a2.run(max_steps=400)
        a2.stop()
    finally:
        ModuleApp._heartbeat = orig
    assert tr2.outputs("temperatureOutput") == []
    assert len(beats) >= 9  # 100 s / HEARTBEAT_S
    gaps = [b - a_ for a_, b in zip(beats, beats[1:])]
    assert max(gaps) <= app_mod.HEARTBEAT_S + 0.5
    assert json.loads(hb.read_text())["messages"] == 2


def test_resnet_module_twin_methods_resume(tmp_path):
    state = str(tmp_path / "state.json")
    tr = FakeTransport({"model": "resnet50", "batch": 1, "report_interval_s": 1.0,
                        "image_size": 64})
    app = ModuleApp(tr, device="cpu", state_path=state, clock=Clock()).start()
    assert tr.reported["status"] == "running" and tr.reported["config"]["batch"] == 1
    app.run(max_steps=6)
    tel = tr.outputs("telemetry")
    assert tel, "telemetry expected every report interval"
    t = tel[-1]
    assert {"images_per_s", "latency_ms", "total_images", "top1", "heartbeat"} <= set(t)
    assert t["images_per_s"] > 0 and t["latency_ms"]["p99"] >= t["latency_ms"]["p50"]
    # twin patch: invalid rejected, valid non-rebuild keeps engine, rebuild key rebuilds
    eng = app.engine
    tr.push_twin_patch({"batch": -5})
    tr.push_twin_patch({"report_interval_s": 2.0})
    app.run(max_steps=1)
    assert "rejected" in tr.reported["lastError"] and app.engine is eng
    tr.push_twin_patch({"batch": 2})
    app.run(max_steps=1)
    assert app.engine is not eng and app.cfg.batch == 2 and app.state["rebuilds"] == 1
    # direct methods
    tr.invoke_method("ping")
    tr.invoke_method("benchmark", {"steps": 2, "warmup": 0})
    tr.invoke_method("getStatus")
    tr.invoke_method("nope")
    app.run(max_steps=1)
    res = {n: (s, r) for n, s, r in tr.method_results}
    assert res["ping"][0] == 200 and res["benchmark"][0] == 200
    assert res["benchmark"][1]["images_per_s"] > 0 and res["benchmark"][1]["batch"] == 2
    assert res["getStatus"][1]["config"]["batch"] == 2 and res["nope"][0] == 404
    total = app.state["total_images"]
    app.stop()
    saved = json.load(open(state))
    assert saved["total_images"] == total and saved["config"]["batch"] == 2
    # restart resumes counters from the persistent disk
    tr2 = FakeTransport({"model": "resnet50", "batch": 1, "image_size": 64})
    app2 = ModuleApp(tr2, device="cpu", state_path=state, clock=Clock()).start()
    assert app2.state["restarts"] == 1 and app2.state["total_images"] == total
    app2.stop()


def test_report_after_auto_report_never_publishes_empty_window():
    """with a short report interval the boundary of the LAST step
    auto-reports (draining the window); an explicit report() right after must carry that
    window (flagged, with its window_s), never publish 0 img/s."""

    class StepClock:  # advances only when told: the test decides when a report is due
        t = 0.0

        def __call__(self):
            return self.t

    clk = StepClock()
    tr = FakeTransport({"model": "resnet50", "batch": 1, "report_interval_s": 0.5,
                        "image_size": 64})
    with ModuleApp(tr, device="cpu", clock=clk).start() as app:
        real_infer = app._infer_step

        def slow_step():  # each step takes 1 s on the fake clock -> every boundary reports
            clk.t += 1.0
            real_infer()

        app._infer_step = slow_step
        app.run(max_steps=3)
        auto = tr.outputs("telemetry")
        assert len(auto) == 3 and auto[-1]["images_per_s"] > 0
        assert auto[-1]["window_carried"] is False
        msg = app.report()  # nothing ran since the last auto-report
        assert msg["images_per_s"] == auto[-1]["images_per_s"] > 0
        assert msg["window_carried"] is True and msg["window_s"] == auto[-1]["window_s"]
        assert tr.outputs("telemetry")[-1]["images_per_s"] > 0
    assert app._closed  # the context manager stopped it
    app.stop()  # idempotent


def test_stdout_transport(capsys):
    tr = StdoutTransport({"model": "simulated-temperature"})
    app = ModuleApp(tr, device="cpu", clock=Clock()).start()
    app.run(max_steps=2)
    lines = [json.loads(l) for l in capsys.readouterr().out.strip().splitlines()]
    assert any("reported" in l for l in lines)
    assert any(l.get("output") == "temperatureOutput" for l in lines)


def test_camera_source_ring_feeds_engine(tmp_path):
    """source="camera": a host producer thread fills the pinned FrameRing and every module
    step consumes one batch from it (CPU: host copy path; GPU: the native serve loop)."""
    from kvedge_amd import ops

    if not ops.load():
        import pytest

        pytest.skip("native runtime not built")
    tr = FakeTransport({"model": "resnet50", "batch": 1, "report_interval_s": 1.0,
                        "image_size": 64, "source": "camera"})
    app = ModuleApp(tr, device="cpu", clock=Clock()).start()
    assert app.ring is not None and app.camera is not None and not app.engine.synthetic
    app.run(max_steps=4)
    tel = tr.outputs("telemetry")
    assert tel and tel[-1]["source"] == "camera" and "frames_dropped" in tel[-1]
    assert app.state["total_images"] == 4 and app.camera.seq >= 4
    tr.push_twin_patch({"source": "synthetic"})  # rebuild key: camera thread stopped
    app.run(max_steps=1)
    assert app.ring is None and app.camera is None and app.engine.synthetic
    app.stop()


def test_failed_rebuild_rolls_back_and_stamps(tmp_path):
    """A rebuild that raises (e.g. batch 4096 exhausts HBM) must not kill the module:
    previous config restored, engine serving, lastError reported.  The first inference
    appends ``module_first_inference`` to the guest boot-timing stamp file."""
    stamps = tmp_path / "boot-timing"
    tr = FakeTransport({"model": "resnet50", "batch": 2, "report_interval_s": 1.0,
                        "image_size": 64})
    app = ModuleApp(tr, device="cpu", clock=Clock(), stamp_path=str(stamps)).start()
    orig = app._build_local

    def build():
        if app.cfg.batch == 4096:
            raise RuntimeError("HIP out of memory (injected)")
        orig()

    app._build_local = build
    app.run(max_steps=2)
    names = [ln.split()[0] for ln in stamps.read_text().splitlines()]
    # the first build's cold-start legs, then the first inference
    assert names == ["module_model_built", "module_tuned", "module_warm",
                     "module_graph_captured", "module_graph_refined", "module_first_inference"]
    eng = app.engine
    tr.push_twin_patch({"batch": 4096})
    app.run(max_steps=1)
    assert app.cfg.batch == 2 and app.engine is not None and app.engine is not eng
    assert "rolled back" in tr.reported["lastError"] and app.state["failed_rebuilds"] == 1
    assert tr.reported["config"]["batch"] == 2 and tr.reported["status"] == "running"
    tr.invoke_method("reconfigure", {"batch": 4096})
    app.run(max_steps=2)
    res = {n: (s, r) for n, s, r in tr.method_results}
    assert res["reconfigure"][0] == 409 and app.cfg.batch == 2
    n0 = app.state["total_images"]
    app.run(max_steps=2)
    assert app.state["total_images"] == n0 + 4  # still serving
    assert stamps.read_text().count("module_first_inference") == 1
    app.stop()


# ------------------------------------------------------------------ stub azure-iot-device
class _StubSdk:
    """Minimal stand-in for azure-iot-device's v2 sync API surface the module uses.
    Records every call in order; a twin patch and a method request are "delivered by
    edgeHub" DURING connect(), i.e. before the module has finished starting."""

    def __init__(self, desired):
        import types

        sdk = self
        self.calls, self.responses, self.sent, self.reported = [], [], [], []
        self.desired = dict(desired, **{"$version": 7})

        class MethodRequest:
            def __init__(self, request_id, name, payload):
                self.request_id, self.name, self.payload = request_id, name, payload

        class Message:
            def __init__(self, data):
                self.data, self.content_type, self.content_encoding = data, None, None

        class MethodResponse:
            def __init__(self, request_id, status, payload):
                self.request_id, self.status, self.payload = request_id, status, payload

            @classmethod
            def create_from_method_request(cls, req, status, payload):
                return cls(req.request_id, status, payload)

        class IoTHubModuleClient:
            def __init__(self):
                self.on_twin_desired_properties_patch_received = None
                self.on_method_request_received = None

            @classmethod
            def create_from_edge_environment(cls):
                sdk.calls.append("create_from_edge_environment")
                sdk.client = cls()
                return sdk.client

            def connect(self):
                sdk.calls.append(("connect",
                                  self.on_twin_desired_properties_patch_received is not None,
                                  self.on_method_request_received is not None))
                # edgeHub pushes these while the connection is coming up
                if self.on_twin_desired_properties_patch_received:
                    self.on_twin_desired_properties_patch_received(
                        {"report_interval_s": 0.5, "$version": 8})
                if self.on_method_request_received:
                    self.on_method_request_received(
                        MethodRequest("r1", "benchmark", {"steps": 1, "warmup": 0}))

            def shutdown(self):
                sdk.calls.append("shutdown")

            def get_twin(self):
                sdk.calls.append("get_twin")
                return {"desired": dict(sdk.desired), "reported": {}}

            def patch_twin_reported_properties(self, props):
                json.dumps(props)  # must be JSON-serialisable
                sdk.reported.append(props)

            def send_message_to_output(self, msg, output):
                sdk.sent.append((output, msg))

            def send_method_response(self, resp):
                sdk.responses.append(resp)

        self.MethodRequest = MethodRequest
        dev = types.ModuleType("azure.iot.device")
        dev.IoTHubModuleClient, dev.Message, dev.MethodResponse = \
            IoTHubModuleClient, Message, MethodResponse
        dev.MethodRequest = MethodRequest
        self.modules = {"azure": types.ModuleType("azure"),
                        "azure.iot": types.ModuleType("azure.iot"), "azure.iot.device": dev}


def test_azure_transport_against_stub_sdk(tmp_path, monkeypatch):
    """the production transport runs end to end through a
    stub ``azure.iot.device``: handlers registered before connect (the patch and method
    sent during connect are not lost), desired twin ($version stripped) -> config,
    deferred ``benchmark`` reply via MethodResponse.create_from_method_request,
    telemetry via send_message_to_output with a JSON content type.  Parity with the
    real SDK is unpinned (the package is not installed in this image)."""
    import sys

    from kvedge_amd.module.transport import make_transport

    sdk = _StubSdk({"model": "resnet50", "batch": 1, "image_size": 64,
                    "report_interval_s": 1000})
    for k, m in sdk.modules.items():
        monkeypatch.setitem(sys.modules, k, m)
    tr = make_transport("azure")
    app = ModuleApp(tr, device="cpu", state_path=str(tmp_path / "s.json"), clock=Clock()).start()
    assert sdk.calls[0] == "create_from_edge_environment"
    assert sdk.calls[1] == ("connect", True, True)  # handlers were already installed
    assert app.cfg.batch == 1 and app.cfg.image_size == 64
    # the deferred method arrived during connect: answered at the first boundary
    app.run(max_steps=3)
    resp = {r.request_id: r for r in sdk.responses}
    assert resp["r1"].status == 200 and resp["r1"].payload["images_per_s"] > 0
    # the patch sent during connect was applied ($version never reaches the config)
    assert app.cfg.report_interval_s == 0.5
    tel = [(o, m) for o, m in sdk.sent if o == "telemetry"]
    assert tel, "telemetry expected after the 0.5 s report interval"
    out, msg = tel[-1]
    assert msg.content_type == "application/json" and msg.content_encoding == "utf-8"
    body = json.loads(msg.data)
    assert body["model"] == "resnet50" and body["images_per_s"] > 0
    assert any(r.get("status") == "running" for r in sdk.reported)
    # a later method through the SDK's handler thread path; unknown -> 404
    sdk.client.on_method_request_received(sdk.MethodRequest("r2", "nope", None))
    sdk.client.on_method_request_received(sdk.MethodRequest("r3", "ping", {}))
    app.run(max_steps=1)
    resp = {r.request_id: r for r in sdk.responses}
    assert resp["r2"].status == 404 and resp["r3"].status == 200
    app.stop()
    assert sdk.calls[-1] == "shutdown"


def test_refine_budget_config():
    """The module's in-graph refine budget is a validated twin/CLI key (0 = off)."""
    import pytest
    from kvedge_amd.module.config import ModuleConfig
    assert ModuleConfig().refine_s == 0.0  # opt-in
    ModuleConfig(refine_s=0.0).validate()
    with pytest.raises(ValueError):
        ModuleConfig(refine_s=-1.0).validate()


def test_module_refuses_cpu_when_gpu_required(tmp_path, capsys, monkeypatch):
    """a GPU VM whose MI355X did not come back must not serve on the CPU.
    With KVEDGE_REQUIRE_GPU (the chart sets it from gpu.count) the module exits non-zero
    with a clear error and writes no heartbeat; without it, the heartbeat names the
    device it runs on, so kvedge-health can tell a CPU fallback apart."""
    import json

    import pytest

    from kvedge_amd.module import __main__ as entry
    from kvedge_amd.module.app import GpuUnavailableError, ModuleApp
    from kvedge_amd.module.transport import FakeTransport

    with pytest.raises(GpuUnavailableError, match="refusing to serve on the CPU"):
        ModuleApp(FakeTransport({"model": "simulated-temperature"}), device="cpu", require_gpus=1)
    hb = tmp_path / "heartbeat"
    monkeypatch.setenv("KVEDGE_REQUIRE_GPU", "1")
    rc = entry.main(["--transport", "fake", "--model", "simulated-temperature", "--steps", "1",
                     "--heartbeat", str(hb), "--state", str(tmp_path / "s.json"),
                     "--stamps", str(tmp_path / "bt"), "--tune-cache", ""])
    assert rc == 3 and not hb.exists()
    assert "refusing to serve on the CPU" in capsys.readouterr().err
    monkeypatch.setenv("KVEDGE_REQUIRE_GPU", "0")
    rc = entry.main(["--transport", "fake", "--model", "simulated-temperature", "--steps", "1",
                     "--heartbeat", str(hb), "--state", str(tmp_path / "s.json"),
                     "--stamps", str(tmp_path / "bt"), "--tune-cache", ""])
    assert rc == 0
    beat = json.loads(hb.read_text())
    assert beat["device"] == "cpu" and beat["gpus"] == 0
