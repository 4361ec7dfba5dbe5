"""IoT Edge module transport abstraction.

The module talks to edgeHub (module twin, telemetry outputs, direct methods).
Three implementations:
  * AzureIoTTransport -- azure-iot-device's IoTHubModuleClient from the IoT Edge
    environment (only inside a real edge runtime; the package is optional and is
    not installed here, so it is imported lazily and fails with a clear message);
  * FakeTransport     -- in-process hub for tests: records messages and reported
    properties, lets tests push twin patches and invoke direct methods;
  * StdoutTransport   -- JSON lines on stdout for bare-metal/bench runs.
"""
from __future__ import annotations

import json
import queue
import sys
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

TwinHandler = Callable[[Dict[str, Any]], None]


class Deferred:
    """A direct-method reply that is produced later.  A multi-replica module answers a
    method that needs collectives (e.g. ``benchmark``) only at the next lockstep
    boundary, when every rank runs it together; IoT Hub keeps the caller waiting until
    the response arrives (up to the method's responseTimeoutInSeconds)."""

    def __init__(self):
        self._result: Optional[Tuple[int, Dict[str, Any]]] = None
        self._sink: Optional[Callable[[int, Dict[str, Any]], None]] = None

    def bind(self, sink: Callable[[int, Dict[str, Any]], None]) -> None:
        self._sink = sink
        if self._result is not None:
            sink(*self._result)

    def resolve(self, status: int, res: Dict[str, Any]) -> None:
        if self._result is not None:
            return
        self._result = (status, res)
        if self._sink is not None:
            self._sink(status, res)

    @property
    def done(self) -> bool:
        return self._result is not None


MethodHandler = Callable[[str, Dict[str, Any]], "Tuple[int, Dict[str, Any]] | Deferred"]


def _deliver(result, sink: Callable[[int, Dict[str, Any]], None]) -> None:
    if isinstance(result, Deferred):
        result.bind(sink)
    else:
        sink(*result)


class Transport:
    def connect(self) -> None:
        pass

    def disconnect(self) -> None:
        pass

    def get_desired(self) -> Dict[str, Any]:
        return {}

    def patch_reported(self, props: Dict[str, Any]) -> None:
        raise NotImplementedError

    def send_message(self, output: str, payload: Dict[str, Any]) -> None:
        raise NotImplementedError

    def set_twin_patch_handler(self, cb: TwinHandler) -> None:
        self._twin_cb = cb

    def set_method_handler(self, cb: MethodHandler) -> None:
        self._method_cb = cb

    def poll(self) -> None:
        """Deliver pending twin patches / method calls on the caller's thread."""


class FakeTransport(Transport):
    """In-process stand-in for edgeHub.  Thread-safe; events are delivered from
    ``poll()`` so the module loop stays single-threaded (no races with the GPU)."""

    def __init__(self, desired: Optional[Dict[str, Any]] = None):
        self.desired: Dict[str, Any] = dict(desired or {})
        self.reported: Dict[str, Any] = {}
        self.messages: List[Tuple[str, Dict[str, Any]]] = []
        self.method_results: List[Tuple[str, int, Dict[str, Any]]] = []
        self.connected = False
        self._events: "queue.Queue" = queue.Queue()
        self._lock = threading.Lock()
        self._twin_cb: Optional[TwinHandler] = None
        self._method_cb: Optional[MethodHandler] = None

    def connect(self):
        self.connected = True

    def disconnect(self):
        self.connected = False

    def get_desired(self):
        with self._lock:
            return dict(self.desired)

    def patch_reported(self, props):
        with self._lock:
            self.reported.update(json.loads(json.dumps(props)))

    def send_message(self, output, payload):
        if not self.connected:
            raise RuntimeError("transport not connected")
        with self._lock:
            self.messages.append((output, json.loads(json.dumps(payload))))

    # --- test-side API ----------------------------------------------------
    def push_twin_patch(self, patch: Dict[str, Any]):
        with self._lock:
            self.desired.update(patch)
        self._events.put(("twin", patch))

    def invoke_method(self, name: str, payload: Optional[Dict[str, Any]] = None):
        self._events.put(("method", (name, payload or {})))

    def poll(self):
        while True:
            try:
                kind, data = self._events.get_nowait()
            except queue.Empty:
                return
            if kind == "twin" and self._twin_cb:
                self._twin_cb(data)
            elif kind == "method" and self._method_cb:
                name = data[0]
                _deliver(self._method_cb(*data),
                         lambda st, res, n=name: self.method_results.append((n, st, res)))

    def outputs(self, name: str) -> List[Dict[str, Any]]:
        with self._lock:
            return [p for o, p in self.messages if o == name]


class NullTransport(Transport):
    """For the non-leader ranks of a multi-GPU VM (topology a): the VM is ONE IoT Edge
    device, so only local rank 0 holds the edgeHub connection; the other ranks take
    part through the lockstep boundaries and have nothing to send."""

    def __init__(self, desired: Optional[Dict[str, Any]] = None):
        self.desired = dict(desired or {})

    def get_desired(self):
        return dict(self.desired)

    def patch_reported(self, props):
        pass

    def send_message(self, output, payload):
        pass


class StdoutTransport(Transport):
    def __init__(self, desired: Optional[Dict[str, Any]] = None, stream=None):
        self.desired = dict(desired or {})
        self.stream = stream or sys.stdout

    def get_desired(self):
        return dict(self.desired)

    def patch_reported(self, props):
        self._emit({"reported": props})

    def send_message(self, output, payload):
        self._emit({"output": output, "payload": payload})

    def _emit(self, obj):
        self.stream.write(json.dumps(obj) + "\n")
        self.stream.flush()


class AzureIoTTransport(Transport):
    """Real edgeHub connection via azure-iot-device (optional dependency; v2 sync API:
    ``IoTHubModuleClient.create_from_edge_environment``, handler properties, ``Message``,
    ``MethodResponse.create_from_method_request``).

    The SDK calls its handlers on its own handler thread; they only enqueue, and
    ``poll()`` delivers on the module thread, so no callback ever races the GPU loop.
    The handlers are installed BEFORE ``connect()``: a desired-properties patch or a
    method request that edgeHub delivers while the connection comes up is queued, not
    dropped.  Tested against a stub SDK in
    tests/test_module_cpu.py; parity with the real package stays unpinned (it is not
    installed in this image).
    """

    def __init__(self, client=None):
        try:
            from azure.iot.device import IoTHubModuleClient, Message, MethodResponse  # noqa
        except ImportError as e:  # pragma: no cover - not installed in CI
            raise RuntimeError(
                "azure-iot-device is not installed; install it in the module image or use "
                "--transport stdout/fake") from e
        self._Message, self._MethodResponse = Message, MethodResponse
        self._events: "queue.Queue" = queue.Queue()
        self._twin_cb: Optional[TwinHandler] = None
        self._method_cb: Optional[MethodHandler] = None
        self.client = client or IoTHubModuleClient.create_from_edge_environment()
        # handlers first: anything edgeHub sends from now on lands in the queue
        self.client.on_twin_desired_properties_patch_received = \
            lambda p: self._events.put(("twin", p))
        self.client.on_method_request_received = lambda r: self._events.put(("method", r))
        self.connected = False

    def connect(self):
        self.client.connect()
        self.connected = True

    def disconnect(self):
        if self.connected:
            self.connected = False
            self.client.shutdown()

    def get_desired(self):
        twin = self.client.get_twin() or {}
        return {k: v for k, v in dict(twin.get("desired", {})).items()
                if not k.startswith("$")}  # $version / $metadata are the hub's

    def patch_reported(self, props):
        self.client.patch_twin_reported_properties(json.loads(json.dumps(props)))

    def send_message(self, output, payload):
        msg = self._Message(json.dumps(payload))
        msg.content_type, msg.content_encoding = "application/json", "utf-8"
        self.client.send_message_to_output(msg, output)

    def _respond(self, req, status: int, res: Dict[str, Any]) -> None:
        self.client.send_method_response(
            self._MethodResponse.create_from_method_request(req, status, res))

    def poll(self):
        while True:
            try:
                kind, data = self._events.get_nowait()
            except queue.Empty:
                return
            if kind == "twin" and self._twin_cb:
                self._twin_cb({k: v for k, v in dict(data).items() if not k.startswith("$")})
            elif kind == "method":
                if self._method_cb is None:
                    self._respond(data, 503, {"error": "module not ready"})
                    continue
                _deliver(self._method_cb(data.name, data.payload or {}),
                         lambda st, res, req=data: self._respond(req, st, res))


def make_transport(kind: str, desired: Optional[Dict[str, Any]] = None) -> Transport:
    if kind == "fake":
        return FakeTransport(desired)
    if kind == "stdout":
        return StdoutTransport(desired)
    if kind == "azure":
        return AzureIoTTransport()
    if kind == "null":
        return NullTransport(desired)
    raise ValueError(f"unknown transport {kind!r}")


def now_iso() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime()) + "Z"
