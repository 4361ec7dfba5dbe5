#!/bin/bash
# Build the pre-baked kvedge guest disk (Ubuntu 24.04 noble) and its containerDisk.
#   deploy/image/build-disk.sh [--push] [TAG]
# Needs on the build host: qemu-img, virt-customize (libguestfs-tools), docker, network.
#
# ROCm userspace lives in the MODULE container (deploy/module); the guest only needs the
# amdgpu kernel driver (amdgpu-dkms) so /dev/kfd and /dev/dri appear for the VFIO-passed
# MI355X, plus moby-engine + aziot-edge.  Everything the reference installs at first boot
# (its four apt operations, _helper.tpl:69-72) is baked here, and the edgeAgent/edgeHub
# images are pre-loaded, so boot-to-`iotedge check` needs no package or image download.
#
# DKMS inside virt-customize: the libguestfs appliance runs ITS OWN kernel, so a plain
# `apt install amdgpu-dkms` builds the module for the appliance kernel, not the guest's.
# The module is therefore built explicitly for the guest kernel found in the image
# (dkms autoinstall -k KVER) and the build FAILS unless `modinfo -k KVER amdgpu` finds it.
set -euo pipefail
cd "$(dirname "$0")"
UBUNTU=${UBUNTU:-noble}
UBUNTU_VER=${UBUNTU_VER:-24.04}
ROCM_REPO=${ROCM_REPO:-https://repo.radeon.com/amdgpu/latest/ubuntu}
SIZE=${SIZE:-30G}
PRELOAD=${PRELOAD:-"mcr.microsoft.com/azureiotedge-agent:1.5 mcr.microsoft.com/azureiotedge-hub:1.5"}
PUSH=0
if [ "${1:-}" = "--push" ]; then PUSH=1; shift; fi
TAG=${1:-ghcr.io/kvedge/ubuntu-rocm-container-disk:${UBUNTU_VER}}
mkdir -p build/images
IMG=build/base.img
[ -f "$IMG" ] || curl -fL -o "$IMG" "https://cloud-images.ubuntu.com/${UBUNTU}/current/${UBUNTU}-server-cloudimg-amd64.img"
cp "$IMG" build/kvedge-guest.qcow2
qemu-img resize build/kvedge-guest.qcow2 "$SIZE"

# edge runtime images, saved on the build host and loaded once at first boot
for ref in $PRELOAD; do
  f="build/images/$(echo "$ref" | tr '/:' '__').tar"
  [ -f "$f" ] || { docker pull "$ref" && docker save -o "$f" "$ref"; }
done

cat > build/kvedge-preload.service <<'UNIT'
[Unit]
Description=kvedge: load pre-baked IoT Edge runtime images (no registry pull at boot)
After=docker.service
Requires=docker.service
Before=aziot-edged.service
ConditionPathExists=!/var/lib/kvedge/images/.loaded
[Service]
Type=oneshot
ExecStart=/bin/sh -c 'for f in /var/lib/kvedge/images/*.tar; do docker load -i "$f"; done && touch /var/lib/kvedge/images/.loaded'
RemainAfterExit=yes
[Install]
WantedBy=multi-user.target
UNIT

virt-customize -a build/kvedge-guest.qcow2 \
  --run-command "growpart /dev/sda 1 || true" \
  --run-command "curl -fsSL https://packages.microsoft.com/config/ubuntu/${UBUNTU_VER}/packages-microsoft-prod.deb -o /tmp/ms.deb && dpkg -i /tmp/ms.deb" \
  --run-command "mkdir -p /etc/apt/keyrings && curl -fsSL https://repo.radeon.com/rocm/rocm.gpg.key | gpg --dearmor -o /etc/apt/keyrings/rocm.gpg" \
  --run-command "echo 'deb [arch=amd64 signed-by=/etc/apt/keyrings/rocm.gpg] ${ROCM_REPO} ${UBUNTU} main' > /etc/apt/sources.list.d/amdgpu.list" \
  --run-command "apt-get update && DEBIAN_FRONTEND=noninteractive apt-get install -y linux-generic moby-engine aziot-edge dkms qemu-guest-agent" \
  --run-command "KVER=\$(ls /lib/modules | sort -V | tail -1) && DEBIAN_FRONTEND=noninteractive apt-get install -y linux-headers-\$KVER && DEBIAN_FRONTEND=noninteractive apt-get install -y --no-install-recommends amdgpu-dkms && dkms autoinstall -k \$KVER && modinfo -k \$KVER amdgpu > /var/log/kvedge-amdgpu-modinfo.txt && echo \$KVER > /etc/kvedge-guest-kernel" \
  --run-command "echo 'blacklist amdgpu_fbdev' > /etc/modprobe.d/kvedge.conf" \
  --mkdir /var/lib/kvedge/images \
  --copy-in build/images:/var/lib/kvedge \
  --copy-in build/kvedge-preload.service:/etc/systemd/system \
  --run-command "systemctl enable docker kvedge-preload.service aziot-edged qemu-guest-agent || true" \
  --run-command "apt-get clean && rm -rf /var/lib/apt/lists/*" \
  --run-command "cloud-init clean --logs || true"
# proof the module exists for the guest kernel (the command above already failed the
# build otherwise); kept next to the image for the release notes
virt-cat -a build/kvedge-guest.qcow2 /var/log/kvedge-amdgpu-modinfo.txt | head -3
qemu-img convert -O qcow2 -c build/kvedge-guest.qcow2 build/kvedge-guest.qcow2.tmp && mv build/kvedge-guest.qcow2.tmp build/kvedge-guest.qcow2
docker build -t "$TAG" .
if [ "$PUSH" = 1 ]; then docker push "$TAG"; fi
echo "containerDisk: docker://$TAG  (set image.containerDisk in deploy/helm/values.yaml)"
