# Round 6 (z13): bench --profile (per-op HIP-event profile) with the updated op list, both models
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z13}
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --edge "" --yolo 0 --profile gpurun_out/${T}_ops_rn.json > gpurun_out/${T}_rn.txt 2>&1 || { tail -20 gpurun_out/${T}_rn.txt; exit 1; }
timeout -k 10 400 python -u bench.py --model yolov8n --steps 3 --warmup 1 --edge "" --profile gpurun_out/${T}_ops_yolo.json > gpurun_out/${T}_yolo.txt 2>&1 || { tail -20 gpurun_out/${T}_yolo.txt; exit 1; }
python - <<'PY'
import json
for m in ("rn", "yolo"):
    d = json.load(open(f"gpurun_out/r6z13_ops_{m}.json"))
    rows = d.get("ops") or d.get("rows") or d
    names = sorted({r.get("op") or r.get("name") for r in rows}) if isinstance(rows, list) else list(rows)[:10]
    print(m, len(rows) if hasattr(rows, "__len__") else "?", names)
PY
