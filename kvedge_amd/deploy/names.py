"""Resource names the chart renders, computed without rendering (for the boot-timing
collector and the resilience KubectlCluster).  Mirrors deploy/helm/templates/_helpers.tpl
(reference naming rule _helper.tpl:6-8: default .Chart.Name .Values.nameOverride |
trunc 40 | trimSuffix "-"; replica i > 0 appends "-<i>").  tests/test_chart.py checks
these against an actual render."""
from __future__ import annotations

CHART_NAME = "aziot-edge-kubevirt"


class ChartNames:
    def __init__(self, name_override: str = CHART_NAME, replicas: int = 1):
        base = (name_override or CHART_NAME)[:40]
        while base.endswith("-"):
            base = base[:-1]
        self.base = base
        self.raw_override = name_override
        self.replicas = replicas

    @staticmethod
    def _sfx(i: int) -> str:
        return f"-{i}" if i > 0 else ""

    def vm(self, i: int = 0) -> str:
        return f"{self.base}-linux{self._sfx(i)}"

    def dv(self, i: int = 0) -> str:
        return f"{self.base}-linux-dv{self._sfx(i)}"

    def domain(self, i: int = 0) -> str:
        return f"{self.base}-vm{self._sfx(i)}"

    def ssh_service(self, i: int = 0) -> str:
        return f"{self.base}-vm-ssh-service{self._sfx(i)}"

    def config_secret(self, i: int = 0) -> str:
        return f"{self.base}-vm-aziotedgeconfig{self._sfx(i)}"

    def cloudinit_secret(self, i: int = 0) -> str:
        # the reference uses the RAW nameOverride here (its TODO, aziot-edge-vm.yaml:57)
        return f"{self.raw_override or self.base}-vm-cloudconfig{self._sfx(i)}"

    def rendezvous(self) -> str:
        return f"{self.base}-dp-rendezvous"

    def all_vms(self):
        return [self.vm(i) for i in range(self.replicas)]
