#!/bin/bash
# Build the pre-baked kvedge guest disk (Ubuntu 24.04 noble) and its containerDisk.
#   deploy/image/build-disk.sh [--push REGISTRY/IMAGE:TAG]
# Needs: qemu-img, virt-customize (libguestfs-tools), docker/podman, network.
# ROCm userspace lives in the MODULE container (deploy/module); the guest only needs
# the amdgpu kernel driver (amdgpu-dkms) so /dev/kfd and /dev/dri appear for the
# VFIO-passed MI355X.
set -euo pipefail
cd "$(dirname "$0")"
UBUNTU=${UBUNTU:-noble}
ROCM_REPO=${ROCM_REPO:-https://repo.radeon.com/amdgpu/latest/ubuntu}
SIZE=${SIZE:-30G}
mkdir -p build
IMG=build/base.img
[ -f "$IMG" ] || curl -fL -o "$IMG" "https://cloud-images.ubuntu.com/${UBUNTU}/current/${UBUNTU}-server-cloudimg-amd64.img"
cp "$IMG" build/kvedge-guest.qcow2
qemu-img resize build/kvedge-guest.qcow2 "$SIZE"
virt-customize -a build/kvedge-guest.qcow2 \
  --run-command "growpart /dev/sda 1 || true" \
  --run-command "curl -fsSL https://packages.microsoft.com/config/ubuntu/24.04/packages-microsoft-prod.deb -o /tmp/ms.deb && dpkg -i /tmp/ms.deb" \
  --run-command "mkdir -p /etc/apt/keyrings && curl -fsSL https://repo.radeon.com/rocm/rocm.gpg.key | gpg --dearmor -o /etc/apt/keyrings/rocm.gpg" \
  --run-command "echo 'deb [arch=amd64 signed-by=/etc/apt/keyrings/rocm.gpg] ${ROCM_REPO} ${UBUNTU} main' > /etc/apt/sources.list.d/amdgpu.list" \
  --run-command "apt-get update && DEBIAN_FRONTEND=noninteractive apt-get install -y moby-engine aziot-edge amdgpu-dkms linux-headers-generic" \
  --run-command "echo 'blacklist amdgpu_fbdev' > /etc/modprobe.d/kvedge.conf" \
  --run-command "systemctl enable docker aziot-edged || true" \
  --run-command "apt-get clean && rm -rf /var/lib/apt/lists/*" \
  --run-command "cloud-init clean --logs || true"
qemu-img convert -O qcow2 -c build/kvedge-guest.qcow2 build/kvedge-guest.qcow2.tmp && mv build/kvedge-guest.qcow2.tmp build/kvedge-guest.qcow2
TAG=${2:-ghcr.io/kvedge/ubuntu-rocm-container-disk:24.04}
docker build -t "$TAG" .
if [ "${1:-}" = "--push" ]; then docker push "$TAG"; fi
echo "containerDisk: docker://$TAG  (set image.containerDisk in deploy/helm/values.yaml)"
