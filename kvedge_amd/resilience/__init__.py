"""N22 resilience: node drain / VM failure -> cold migration with MI355X re-attach.

What the reference offers: the VirtualMachine's
`running: true` makes KubeVirt recreate a dead VMI; the PVC keeps EdgeHub state; a
static MAC keeps NIC identity; but an RWO PVC pins the VM to its node, so cross-node
recovery fails (reference README.md:89), and nothing handles eviction.

kvedge adds, for VMs with VFIO-passed GPUs (which KubeVirt cannot live-migrate):
  * a controller that turns drain / node loss / GPU failure into a COLD migration:
    stop the VMI, release its GPUs, pick a node with free MI355X capacity whose storage
    can attach the boot PVC (RWX anywhere, RWO only on its bound node), start it,
    re-attach GPUs, wait for the module heartbeat -- with a per-phase timeline;
  * the same state machine against a fake, dict-backed cluster (tests, fault injection)
    and a KubectlAdapter that emits the equivalent kubectl/virtctl commands
    (dry-run by default; there is no cluster in CI).
"""
from __future__ import annotations

import subprocess
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

RWO, RWX = "ReadWriteOnce", "ReadWriteMany"


@dataclass
class Timings:
    """Seconds per phase of a cold migration, fed to the FakeCluster's clock.

    The defaults are ASSUMED INPUTS, not measurements (no cluster has been run): any
    "cold-migration time" computed from them is a model output and is labelled
    ``source="assumed"``.  :meth:`from_boot_summary` replaces the guest-side phases with
    the ones the boot-timing collector measured (kvedge_amd.utils.boottime collect)."""
    graceful_stop: float = 20.0
    node_failure_detect: float = 40.0
    schedule: float = 2.0
    pvc_attach: float = 8.0
    gpu_attach: float = 3.0
    guest_boot: float = 45.0
    module_ready: float = 15.0
    source: str = "assumed"

    @classmethod
    def from_boot_summary(cls, summary: Dict[str, float],
                          base: Optional["Timings"] = None) -> "Timings":
        """Derive the boot phases from one replica's collector summary (seconds after
        helm install): guest_boot = VMI Running -> cloud-init runcmd done (includes the
        GPU wait); module_ready = runcmd done -> ready (iotedge check pass, else the
        module's first inference).  Phases the summary lacks keep ``base``'s values."""
        b = base or cls()
        kw = dict(b.__dict__)
        run, done = summary.get("vmi_running_s"), summary.get("guest_runcmd_done_s")
        ready = summary.get("iotedge_check_pass_s", summary.get("module_first_inference_s"))
        measured = []
        if run is not None and done is not None and done >= run:
            kw["guest_boot"] = done - run
            measured.append("guest_boot")
        if done is not None and ready is not None and ready >= done:
            kw["module_ready"] = ready - done
            measured.append("module_ready")
        kw["source"] = ("boot-timing:" + ",".join(measured)) if measured else b.source
        return cls(**kw)


@dataclass
class Node:
    name: str
    gpus: List[str]
    ready: bool = True
    schedulable: bool = True
    used: Dict[str, str] = field(default_factory=dict)  # gpu id -> vm name

    def free_gpus(self) -> List[str]:
        return [g for g in self.gpus if g not in self.used]


@dataclass
class PVC:
    name: str
    access_mode: str = RWO
    bound_node: Optional[str] = None


@dataclass
class VM:
    name: str
    pvc: str
    gpus: int = 1
    run_strategy: str = "Always"
    host_devices: bool = True


@dataclass
class VMI:
    vm: str
    node: str
    gpu_ids: List[str]
    phase: str = "Running"


@dataclass
class Event:
    t: float
    vm: str
    what: str
    detail: str = ""


class FakeCluster:
    """Dict-backed KubeVirt-ish cluster with a simulated clock and fault injection."""

    def __init__(self, timings: Optional[Timings] = None):
        self.nodes: Dict[str, Node] = {}
        self.pvcs: Dict[str, PVC] = {}
        self.vms: Dict[str, VM] = {}
        self.vmis: Dict[str, VMI] = {}
        self.t = 0.0
        self.timings = timings or Timings()
        self.events: List[Event] = []

    def log(self, vm, what, detail=""):
        self.events.append(Event(self.t, vm, what, detail))

    def advance(self, dt: float):
        self.t += dt

    # --- objects -------------------------------------------------------------
    def add_node(self, name: str, n_gpus: int):
        self.nodes[name] = Node(name, [f"{name}/gpu{i}" for i in range(n_gpus)])

    def add_vm(self, name: str, gpus: int = 1, access_mode: str = RWO):
        self.pvcs[name + "-dv"] = PVC(name + "-dv", access_mode)
        self.vms[name] = VM(name, name + "-dv", gpus)

    # --- scheduling ----------------------------------------------------------
    def candidates(self, vm: VM, exclude: Tuple[str, ...] = ()) -> Tuple[List[str], str]:
        pvc = self.pvcs[vm.pvc]
        out, reasons = [], []
        for n in self.nodes.values():
            if n.name in exclude:
                continue
            if not (n.ready and n.schedulable):
                reasons.append(f"{n.name}: not ready/cordoned")
                continue
            if len(n.free_gpus()) < vm.gpus:
                reasons.append(f"{n.name}: {len(n.free_gpus())} free MI355X < {vm.gpus}")
                continue
            if pvc.access_mode == RWO and pvc.bound_node not in (None, n.name):
                reasons.append(f"{n.name}: RWO PVC {pvc.name} bound to {pvc.bound_node}")
                continue
            out.append(n.name)
        return out, "; ".join(reasons)

    def start(self, vm_name: str, exclude: Tuple[str, ...] = ()) -> Optional[VMI]:
        vm = self.vms[vm_name]
        cands, why = self.candidates(vm, exclude)
        if not cands:
            self.log(vm_name, "unschedulable", why)
            return None
        # prefer the node already holding the PVC (no re-attach), then most free GPUs
        pvc = self.pvcs[vm.pvc]
        cands.sort(key=lambda n: (n != pvc.bound_node, -len(self.nodes[n].free_gpus()), n))
        node = self.nodes[cands[0]]
        tm = self.timings
        self.advance(tm.schedule)
        self.log(vm_name, "scheduled", node.name)
        if pvc.bound_node != node.name:
            self.advance(tm.pvc_attach)
            pvc.bound_node = node.name
            self.log(vm_name, "pvc_attached", node.name)
        ids = node.free_gpus()[:vm.gpus]
        for g in ids:
            node.used[g] = vm_name
        self.advance(tm.gpu_attach)
        self.log(vm_name, "gpu_attached", ",".join(ids))
        self.advance(tm.guest_boot)
        vmi = VMI(vm_name, node.name, ids)
        self.vmis[vm_name] = vmi
        self.log(vm_name, "running", node.name)
        self.advance(tm.module_ready)
        self.log(vm_name, "module_ready", node.name)
        return vmi

    def stop(self, vm_name: str, graceful: bool = True):
        vmi = self.vmis.pop(vm_name, None)
        if vmi is None:
            return
        node = self.nodes[vmi.node]
        for g in vmi.gpu_ids:
            node.used.pop(g, None)
        if graceful:
            self.advance(self.timings.graceful_stop)
        self.log(vm_name, "stopped", vmi.node)

    # --- fault injection -----------------------------------------------------
    def kill_vmi(self, vm_name: str):
        self.stop(vm_name, graceful=False)
        self.log(vm_name, "fault", "vmi killed")

    def node_down(self, node: str):
        self.nodes[node].ready = False
        for name, vmi in list(self.vmis.items()):
            if vmi.node == node:
                self.stop(name, graceful=False)
                self.log(name, "fault", f"node {node} lost")
        self.advance(self.timings.node_failure_detect)

    def gpu_failure(self, gpu_id: str):
        node = self.nodes[gpu_id.split("/")[0]]
        vm = node.used.get(gpu_id)
        node.gpus.remove(gpu_id)
        if vm:
            self.stop(vm, graceful=False)
            self.log(vm, "fault", f"gpu {gpu_id} failed")


@dataclass
class Recovery:
    vm: str
    ok: bool
    from_node: Optional[str]
    to_node: Optional[str]
    seconds: float
    live_migration_refused: bool = False
    reason: str = ""
    gpu_ids: List[str] = field(default_factory=list)


class ResilienceController:
    """Reconciles VMs with runStrategy Always; implements drain as cold migration."""

    def __init__(self, cluster: FakeCluster):
        self.c = cluster

    def reconcile(self) -> List[Recovery]:
        out = []
        for name, vm in self.c.vms.items():
            if vm.run_strategy == "Always" and name not in self.c.vmis:
                t0 = self.c.t
                vmi = self.c.start(name)
                out.append(Recovery(name, vmi is not None, None, vmi.node if vmi else None,
                                    self.c.t - t0, reason="" if vmi else self._why(name),
                                    gpu_ids=vmi.gpu_ids if vmi else []))
        return out

    def _why(self, name):
        evs = [e for e in self.c.events if e.vm == name and e.what == "unschedulable"]
        return evs[-1].detail if evs else ""

    def drain(self, node_name: str, request_live_migration: bool = True) -> List[Recovery]:
        node = self.c.nodes[node_name]
        node.schedulable = False  # cordon
        res = []
        for name, vmi in list(self.c.vmis.items()):
            if vmi.node != node_name:
                continue
            vm = self.c.vms[name]
            refused = request_live_migration and vm.host_devices
            if refused:
                self.c.log(name, "live_migration_refused", "VFIO host devices are not migratable")
            t0 = self.c.t
            self.c.stop(name, graceful=True)
            new = self.c.start(name)
            res.append(Recovery(name, new is not None, node_name, new.node if new else None,
                                self.c.t - t0, refused, "" if new else self._why(name),
                                new.gpu_ids if new else []))
        return res

    def recover_node_loss(self, node_name: str) -> List[Recovery]:
        victims = [n for n, v in self.c.vmis.items() if v.node == node_name]
        t0 = self.c.t
        self.c.node_down(node_name)
        res = []
        for name in victims:
            new = self.c.start(name)
            res.append(Recovery(name, new is not None, node_name, new.node if new else None,
                                self.c.t - t0, reason="" if new else self._why(name),
                                gpu_ids=new.gpu_ids if new else []))
        return res

    def timeline(self, vm: str) -> List[Tuple[float, str, str]]:
        return [(e.t, e.what, e.detail) for e in self.c.events if e.vm == vm]


class KubectlAdapter:
    """The same operations against a real cluster (kubectl + virtctl).  dry_run=True
    returns the command lines without executing them.  VM names come from
    :class:`kvedge_amd.deploy.names.ChartNames` (checked against a chart render in
    tests/test_resilience.py)."""

    def __init__(self, namespace: str = "default", dry_run: bool = True):
        self.ns = namespace
        self.dry_run = dry_run
        self.log: List[List[str]] = []

    def _run(self, *cmd: str) -> str:
        self.log.append(list(cmd))
        if self.dry_run:
            return ""
        return subprocess.run(list(cmd), check=True, capture_output=True, text=True).stdout

    def drain_node(self, node: str):
        self._run("kubectl", "cordon", node)
        # VFIO VMIs refuse live migration: stop them explicitly so the VM controller
        # (runStrategy Always) reschedules them cold on another node
        self._run("kubectl", "drain", node, "--ignore-daemonsets", "--delete-emptydir-data",
                  "--pod-selector=kubevirt.io=virt-launcher", "--timeout=300s")

    def restart_vm(self, vm: str):
        self._run("virtctl", "restart", vm, "-n", self.ns)

    def stop_vm(self, vm: str):
        self._run("virtctl", "stop", vm, "-n", self.ns)

    def start_vm(self, vm: str):
        self._run("virtctl", "start", vm, "-n", self.ns)

    def wait_running(self, vm: str, timeout_s: int = 600):
        self._run("kubectl", "wait", f"vmi/{vm}", "-n", self.ns, "--for=jsonpath={.status.phase}=Running",
                  f"--timeout={timeout_s}s")

    def uncordon(self, node: str):
        self._run("kubectl", "uncordon", node)

    def wait_deleted(self, vm: str, timeout_s: int = 300):
        self._run("kubectl", "wait", f"vmi/{vm}", "-n", self.ns, "--for=delete",
                  f"--timeout={timeout_s}s")

    def cold_migrate(self, vm: str, from_node: str, timeout_s: int = 600):
        """Drain one node's GPU VM the only way VFIO allows: cordon, stop (releases the
        MI355X), wait until the VMI is gone, start (scheduler picks a node with a free
        GPU; RWX storage lets it leave the node), wait Running; uncordon is left to the
        operator after maintenance."""
        self._run("kubectl", "cordon", from_node)
        self.stop_vm(vm)
        self.wait_deleted(vm)
        self.start_vm(vm)
        self.wait_running(vm, timeout_s)
