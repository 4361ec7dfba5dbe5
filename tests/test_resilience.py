"""T-resilience: drain / node loss / GPU failure on a fake cluster."""
from kvedge_amd.resilience import (RWO, RWX, FakeCluster, KubectlAdapter, ResilienceController,
                                   Timings)


def _cluster(access=RWO, nodes=(("n1", 8), ("n2", 8)), vms=2):
    c = FakeCluster(Timings())
    for n, g in nodes:
        c.add_node(n, g)
    for i in range(vms):
        c.add_vm(f"vm{i}", gpus=1, access_mode=access)
    ctl = ResilienceController(c)
    return c, ctl


def test_initial_reconcile_places_all_vms_with_gpus():
    c, ctl = _cluster(nodes=(("n1", 8),))
    rec = ctl.reconcile()
    assert all(r.ok for r in rec) and len(c.vmis) == 2
    used = [g for v in c.vmis.values() for g in v.gpu_ids]
    assert len(set(used)) == 2  # distinct MI355X per VM


def test_drain_rwo_blocks_cross_node_recovery_like_reference():
    c, ctl = _cluster(access=RWO)
    ctl.reconcile()
    node = c.vmis["vm0"].node
    rec = ctl.drain(node)
    assert rec and all(not r.ok for r in rec)
    assert all(r.live_migration_refused for r in rec)
    assert "RWO PVC" in rec[0].reason  # reference README.md:89 limitation, detected


def test_drain_rwx_cold_migrates_with_gpu_reattach():
    c, ctl = _cluster(access=RWX)
    ctl.reconcile()
    src = c.vmis["vm0"].node
    old_gpu = c.vmis["vm0"].gpu_ids
    rec = {r.vm: r for r in ctl.drain(src)}
    r = rec["vm0"]
    assert r.ok and r.to_node != src and r.gpu_ids and r.gpu_ids != old_gpu
    tl = [w for _, w, _ in ctl.timeline("vm0")]
    i = tl.index("live_migration_refused")
    assert tl[i:i + 7] == ["live_migration_refused", "stopped", "scheduled", "pvc_attached",
                           "gpu_attached", "running", "module_ready"]
    tm = c.timings
    assert r.seconds == tm.graceful_stop + tm.schedule + tm.pvc_attach + tm.gpu_attach + \
        tm.guest_boot + tm.module_ready
    assert not c.nodes[src].used  # GPUs released on the drained node


def test_two_vms_one_node_gpu_failure_reattaches_spare():
    """BASELINE config 5: 2 VMs on one 8x MI355X node; a GPU dies -> VM restarts on a spare."""
    c, ctl = _cluster(access=RWO, nodes=(("n1", 8),))
    ctl.reconcile()
    failed = c.vmis["vm1"].gpu_ids[0]
    c.gpu_failure(failed)
    rec = ctl.reconcile()
    assert len(rec) == 1 and rec[0].ok and rec[0].to_node == "n1"
    assert failed not in rec[0].gpu_ids
    assert len(c.nodes["n1"].gpus) == 7


def test_node_loss_and_capacity_limits():
    c, ctl = _cluster(access=RWX, nodes=(("n1", 2), ("n2", 1)), vms=3)
    ctl.reconcile()
    placed = {v: c.vmis[v].node for v in c.vmis}
    assert sorted(placed.values()).count("n1") == 2
    rec = ctl.recover_node_loss("n1")
    oks = [r for r in rec if r.ok]
    fails = [r for r in rec if not r.ok]
    assert len(oks) == 0 and len(fails) == 2  # n2's only GPU is taken
    assert "free MI355X" in fails[0].reason
    c.nodes["n1"].ready = True
    rec2 = ctl.reconcile()
    assert all(r.ok for r in rec2) and len(c.vmis) == 3


def test_kubectl_adapter_dry_run():
    k = KubectlAdapter("edge", dry_run=True)
    k.drain_node("n1")
    k.restart_vm("aziot-edge-kubevirt-linux")
    k.wait_running("aziot-edge-kubevirt-linux")
    k.uncordon("n1")
    cmds = [" ".join(c) for c in k.log]
    assert cmds[0] == "kubectl cordon n1"
    assert cmds[1].startswith("kubectl drain n1")
    assert cmds[2] == "virtctl restart aziot-edge-kubevirt-linux -n edge"
    assert "--for=jsonpath={.status.phase}=Running" in cmds[3]
