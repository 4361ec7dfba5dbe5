{{/*
kvedge chart helpers.  Resource names of replica 0 are exactly the reference's
(levi106/kvedge _helper.tpl:6-8 naming rule: default .Chart.Name .Values.nameOverride,
trunc 40, trimSuffix "-"); replica i>0 appends "-<i>".
*/}}

{{- define "kvedge.name" -}}
{{- default .Chart.Name .Values.nameOverride | trunc 40 | trimSuffix "-" -}}
{{- end -}}

{{- define "kvedge.chart" -}}
{{- printf "%s-%s" .Chart.Name .Chart.Version | replace "+" "_" | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{/* "" for replica 0, "-<i>" otherwise.  Context: (dict "root" $ "i" $i) */}}
{{- define "kvedge.sfx" -}}
{{- if gt (int .i) 0 }}-{{ .i }}{{ end -}}
{{- end -}}

{{/* Common labels (reference emitted version + managed-by; we add the chart label
     the reference defined but never used, plus instance/part-of). */}}
{{- define "kvedge.labels" -}}
helm.sh/chart: {{ include "kvedge.chart" . }}
{{- if .Chart.AppVersion }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
{{- end }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/part-of: kvedge
{{- end -}}

{{/* Bool-or-string flag, e.g. --set-string aziotEdgeVmEnableExternalSsh=true. */}}
{{- define "kvedge.flag" -}}
{{- if eq (lower (toString .)) "true" }}true{{ end -}}
{{- end -}}

{{/* Per-replica names.  Context: (dict "root" $ "i" $i) */}}
{{- define "kvedge.vmName" -}}{{ include "kvedge.name" .root }}-linux{{ include "kvedge.sfx" . }}{{- end -}}
{{- define "kvedge.dvName" -}}{{ include "kvedge.name" .root }}-linux-dv{{ include "kvedge.sfx" . }}{{- end -}}
{{- define "kvedge.domain" -}}{{ include "kvedge.name" .root }}-vm{{ include "kvedge.sfx" . }}{{- end -}}
{{- define "kvedge.svcName" -}}{{ include "kvedge.name" .root }}-vm-ssh-service{{ include "kvedge.sfx" . }}{{- end -}}
{{- define "kvedge.cfgSecret" -}}{{ include "kvedge.name" .root }}-vm-aziotedgeconfig{{ include "kvedge.sfx" . }}{{- end -}}
{{/* The reference names the cloud-init Secret from the RAW nameOverride (its TODO
     at aziot-edge-vm.yaml:57).  Same name whenever nameOverride is set; falls back to
     the truncated name instead of the invalid "-vm-cloudconfig" when it is empty. */}}
{{- define "kvedge.ciSecret" -}}{{ default (include "kvedge.name" .root) .root.Values.nameOverride }}-vm-cloudconfig{{ include "kvedge.sfx" . }}{{- end -}}

{{/* Multi-VM data parallelism active: dp.enabled and more than one VM. */}}
{{- define "kvedge.dpActive" -}}
{{- if and .Values.dp.enabled (gt (int .Values.replicas) 1) }}true{{ end -}}
{{- end -}}
{{- define "kvedge.rdzvName" -}}{{ include "kvedge.name" . }}-dp-rendezvous{{- end -}}
{{/* ranks per VM (one per passed-through GPU, at least 1) */}}
{{- define "kvedge.ranksPerVm" -}}{{ max 1 (int .Values.gpu.count) }}{{- end -}}

{{- define "kvedge.replicaConfig" -}}
{{- $cfgs := .root.Values.replicaConfigs | default list -}}
{{- if lt (int .i) (len $cfgs) }}{{ index $cfgs (int .i) }}{{ else }}{{ .root.Values.azIotEdgeConfig }}{{ end -}}
{{- end -}}

{{/* Secret-disk serial: the bootcmd mount and the VM disk must agree (reference
     aziot-edge-vm.yaml:28 / _helper.tpl:64). */}}
{{- define "kvedge.secretSerial" -}}D23YZ9W6WA5DJ487{{- end -}}

{{/*
cloud-init user-data (GPU-aware).  Context: (dict "root" $ "i" $i)
 * same contract as the reference: secret disk (found by serial) mounted at
   /mnt/app-secret, its `userdata` installed as /etc/aziot/config.toml, then
   `iotedge config apply`;
 * but idempotent on EVERY boot (systemd oneshot comparing contents), so a
   `helm upgrade --set-file azIotEdgeConfig=...` + VM restart rotates the config;
 * nothing is installed when the image is pre-baked (no apt on the boot path);
 * waits for the passed-through MI355X (/dev/kfd, /dev/dri/renderD*) and records
   boot-timing stamps for the boot-to-ready metric (kvedge_amd/utils/boottime.py).
*/}}
{{- define "kvedge.cloudinit" -}}
{{- $v := .root.Values -}}
#cloud-config
hostname: {{ $v.guest.hostname }}{{ include "kvedge.sfx" . }}
{{- if $v.publicSshKey }}
ssh_authorized_keys:
  - {{ $v.publicSshKey }}
{{- end }}
{{- if not $v.image.prebaked }}
apt:
  sources:
    microsoft-prod.list:
      source: "deb [arch=amd64] https://packages.microsoft.com/ubuntu/{{ $v.guest.ubuntuVersion }}/prod {{ $v.guest.ubuntuCodename }} main"
      keyid: BC528686B50D79E339D3721CEB3E94ADBE1229CF
{{- end }}
bootcmd:
  - [sh, -c, "mkdir -p /mnt/app-secret /var/lib/kvedge && echo \"bootcmd $(date +%s.%N) $(cat /proc/sys/kernel/random/boot_id)\" >> /var/lib/kvedge/boot-timing"]
  - [sh, -c, "mountpoint -q /mnt/app-secret || mount -o ro /dev/disk/by-id/virtio-{{ include "kvedge.secretSerial" . }} /mnt/app-secret || mount -o ro /dev/$(lsblk -dno NAME,SERIAL | awk '$2==\"{{ include "kvedge.secretSerial" . }}\"{print $1}') /mnt/app-secret"]
write_files:
  - path: /usr/local/sbin/kvedge-stamp
    permissions: "0755"
    content: |
      #!/bin/sh
      # "<name> <epoch> <boot id>": the boot id scopes a stamp to one boot (the file is on
      # the persistent boot disk and keeps every boot's stamps for the collector)
      mkdir -p /var/lib/kvedge
      echo "$1 $(date +%s.%N) $(cat /proc/sys/kernel/random/boot_id 2>/dev/null)" >> /var/lib/kvedge/boot-timing
  - path: /usr/local/sbin/kvedge-apply-config
    permissions: "0755"
    content: |
      #!/bin/sh
      # Apply /mnt/app-secret/userdata as the IoT Edge config.  Safe on every boot.
      # The new file is staged and only moved to /etc/aziot/config.toml AFTER
      # `iotedge config apply` accepted it; the applied content's hash is recorded, so
      # a failed apply (iotedge not ready yet) is retried on the next run instead of
      # being skipped because the destination already matches.
      set -eu
      src=/mnt/app-secret/userdata
      dst=/etc/aziot/config.toml
      mark=/var/lib/kvedge/config.applied
      [ -s "$src" ] || { echo "kvedge: no config on secret disk"; exit 0; }
      mkdir -p /etc/aziot /var/lib/kvedge
      want=$(sha256sum "$src" | cut -d' ' -f1)
      if [ -f "$mark" ] && [ "$(cat "$mark")" = "$want" ] && [ -f "$dst" ]; then
        /usr/local/sbin/kvedge-stamp config_applied
        exit 0
      fi
      command -v iotedge >/dev/null 2>&1 || { echo "kvedge: iotedge not installed yet"; exit 1; }
      tmp="$dst.kvedge-new"
      install -m 0600 "$src" "$tmp"
      if ! iotedge config apply -c "$tmp"; then
        rm -f "$tmp"
        echo "kvedge: iotedge config apply failed; will retry"
        exit 1
      fi
      mv -f "$tmp" "$dst"
      echo "$want" > "$mark"
      /usr/local/sbin/kvedge-stamp config_applied
  - path: /usr/local/sbin/kvedge-gpu-check
    permissions: "0755"
    content: |
      #!/bin/sh
      # Wait for the VFIO-passed MI355X to be bound by amdgpu inside the guest.  Runs on
      # EVERY boot (kvedge-gpu.service), so gpu.json and the gpu_ready / gpu_missing stamp
      # describe this boot: after a cold migration the re-attached GPU is proven here, not
      # by the scheduler's allocation.
      want=${1:-1}; wait_s=${2:-120}; t=0; n=0
      boot=$(cat /proc/sys/kernel/random/boot_id 2>/dev/null)
      mkdir -p /var/lib/kvedge
      while [ "$t" -lt "$wait_s" ]; do
        n=$(ls /dev/dri/renderD* 2>/dev/null | wc -l)
        if [ "$want" -eq 0 ] || { [ -e /dev/kfd ] && [ "$n" -ge "$want" ]; }; then
          echo "{\"kfd\": $([ -e /dev/kfd ] && echo true || echo false), \"render_nodes\": $n, \"wanted\": $want, \"waited_s\": $t, \"boot_id\": \"$boot\"}" > /var/lib/kvedge/gpu.json
          /usr/local/sbin/kvedge-stamp gpu_ready
          exit 0
        fi
        sleep 1; t=$((t+1))
      done
      echo "{\"kfd\": $([ -e /dev/kfd ] && echo true || echo false), \"render_nodes\": $n, \"wanted\": $want, \"waited_s\": $t, \"boot_id\": \"$boot\", \"error\": \"timeout\"}" > /var/lib/kvedge/gpu.json
      /usr/local/sbin/kvedge-stamp gpu_missing
      exit 1
  - path: /usr/local/sbin/kvedge-ready
    permissions: "0755"
    content: |
      #!/bin/sh
      # Boot-to-ready producer: poll `iotedge list` until edgeAgent runs and
      # `iotedge check` until it passes (exit 0 = no failed check; warnings allowed),
      # bounded; stamp both into /var/lib/kvedge/boot-timing and keep the last check
      # report as JSON for the collector (python -m kvedge_amd.utils.boottime collect).
      wait_s=${1:-900}; poll_s=${2:-2}; t0=$(date +%s); agent=0
      mkdir -p /var/lib/kvedge
      while [ $(( $(date +%s) - t0 )) -lt "$wait_s" ]; do
        if [ "$agent" -eq 0 ] && iotedge list 2>/dev/null | awk '$1=="edgeAgent" && $2=="running"{f=1} END{exit !f}'; then
          /usr/local/sbin/kvedge-stamp edge_agent_running; agent=1
        fi
        if iotedge check --output json > /var/lib/kvedge/iotedge-check.json 2>/dev/null; then
          [ "$agent" -eq 1 ] || /usr/local/sbin/kvedge-stamp edge_agent_running
          /usr/local/sbin/kvedge-stamp iotedge_check_pass
          exit 0
        fi
        sleep "$poll_s"
      done
      /usr/local/sbin/kvedge-stamp iotedge_check_timeout
      exit 1
  - path: /usr/local/sbin/kvedge-health
    permissions: "0755"
    content: |
      #!/bin/sh
      # VMI probe (guest-agent exec).  Evidence counts only if THIS boot wrote it: the
      # heartbeat and boot-timing live on the persistent boot disk, so a previous boot's
      # fresh heartbeat or iotedge_check_pass line must not make a restarted VMI Ready.
      #   ready = this boot's module heartbeat is fresh (or, with no module, this boot's
      #           iotedge check passed); with gpu.count > 0 also this boot's gpu_ready
      #           stamp and a heartbeat from a module serving on the GPU
      #   live  = no STALE heartbeat of this boot (none yet, or a previous boot's: booting)
      hb=/var/lib/kvedge/heartbeat; bt=/var/lib/kvedge/boot-timing; max={{ $v.health.heartbeatMaxAgeS }}
      boot=$(cat /proc/sys/kernel/random/boot_id 2>/dev/null)
      age() { echo $(( $(date +%s) - $(stat -c %Y "$hb") )); }
      this_boot() { [ -n "$boot" ] && [ -f "$hb" ] && grep -qF "\"boot_id\": \"$boot\"" "$hb"; }
      stamped() { [ -n "$boot" ] && awk -v s="$1" -v b="$boot" '$1==s && $3==b {f=1} END{exit !f}' "$bt" 2>/dev/null; }
      {{- if gt (int $v.gpu.count) 0 }}
      gpu_ok() { stamped gpu_ready; }
      module_gpu() { grep -qF '"device": "cuda"' "$hb"; }
      {{- else }}
      gpu_ok() { true; }
      module_gpu() { true; }
      {{- end }}
      case "$1" in
        ready)
      {{- if $v.module.enabled }}
          this_boot && [ "$(age)" -le "$max" ] && gpu_ok && module_gpu ;;
      {{- else }}
          stamped iotedge_check_pass && gpu_ok ;;
      {{- end }}
        live)
          ! this_boot || [ "$(age)" -le "$max" ] ;;
        *) exit 2 ;;
      esac
  - path: /etc/systemd/system/kvedge-config.service
    content: |
      [Unit]
      Description=kvedge: apply IoT Edge config.toml from the secret disk
      After=local-fs.target network-online.target
      Wants=network-online.target
      [Service]
      Type=oneshot
      ExecStart=/usr/local/sbin/kvedge-apply-config
      RemainAfterExit=yes
      Restart=on-failure
      RestartSec=5
      [Install]
      WantedBy=multi-user.target
  - path: /etc/systemd/system/kvedge-gpu.service
    content: |
      [Unit]
      Description=kvedge: wait for the passed-through MI355X on every boot (gpu_ready stamp)
      After=systemd-modules-load.service systemd-udev-settle.service
      Before=aziot-edged.service kvedge-ready.service
      [Service]
      Type=oneshot
      ExecStart=/usr/local/sbin/kvedge-gpu-check {{ $v.gpu.count }} {{ $v.guest.gpuWaitSeconds }}
      RemainAfterExit=yes
      [Install]
      WantedBy=multi-user.target
  - path: /etc/systemd/system/kvedge-ready.service
    content: |
      [Unit]
      Description=kvedge: wait for iotedge check to pass (boot-to-ready stamp)
      After=kvedge-config.service aziot-edged.service
      Wants=kvedge-config.service
      [Service]
      Type=oneshot
      ExecStart=/usr/local/sbin/kvedge-ready {{ $v.guest.readyWaitSeconds }} {{ $v.guest.readyPollSeconds }}
      RemainAfterExit=yes
      [Install]
      WantedBy=multi-user.target
runcmd:
{{- if not $v.image.prebaked }}
  - [sh, -c, "apt-get update && apt-get install -y moby-engine && apt-get install -y aziot-edge"]
{{- end }}
  - [sh, -c, "getent group render >/dev/null && getent passwd iotedge >/dev/null && usermod -aG video,render iotedge || true"]
  - [systemctl, daemon-reload]
  - [systemctl, enable, --now, kvedge-config.service]
  - [systemctl, enable, --now, --no-block, kvedge-ready.service]
{{- if $v.health.enabled }}
  # exec probes run through the QEMU guest agent (pre-baked; apt only without the image)
  - [sh, -c, "command -v qemu-ga >/dev/null || {{ if $v.image.prebaked }}true{{ else }}apt-get install -y qemu-guest-agent{{ end }}; systemctl enable --now qemu-guest-agent || true"]
{{- end }}
  - [systemctl, enable, --now, kvedge-gpu.service]
  - [/usr/local/sbin/kvedge-stamp, runcmd_done]
final_message: "kvedge guest {{ $v.guest.hostname }}{{ include "kvedge.sfx" . }} up after $UPTIME s"
{{- end -}}
