"""kvedge_amd — MI355X-native IoT-Edge-on-Kubernetes inference framework.

Capabilities of levi106/kvedge (Helm/KubeVirt/CDI/cloud-init deployment of Azure
IoT Edge) re-designed MI355X-first, plus the north-star GPU inference path:
hand-written CDNA4 HIP kernels (gfx950), ResNet-50 / YOLOv8n edge modules, hipGraph
engine and RCCL data parallelism.  See SURVEY.md for the blueprint.
"""
__version__ = "0.2.0"
