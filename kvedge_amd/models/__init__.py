"""Model zoo: ResNet-50 v1.5 and YOLOv8n (random-init, seeded; BN folded; NHWC bf16)."""
from .resnet import KvResNet50, ResNet50Ref, init_resnet50  # noqa: F401
