#!/bin/bash
# train.py on synthetic JPEG pairs (the real input path: DataLoader workers
# decode, one packed H2D copy + one resize/normalise launch per batch), one GPU,
# as a plain process and under torchrun --nproc-per-node 1 (RCCL process
# group, world 1) -> gpurun_out/$REAL_TAG/{plain,torchrun}.log + summary.json
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${REAL_TAG:-r5_real}"
mkdir -p "$OUT"
D=/tmp/ncnet_jpeg_pairs
python3 "$ROOT/scripts/make_jpeg_pairs.py" --out "$D" --pairs 1200 || exit $?
COMMON="--dataset_image_path $D --dataset_csv_path $D/image_pairs --max_steps 150 --log_interval 50 --result-model-dir /tmp/ncnet_ckpt"
timeout -k 10 400 python3 "$ROOT/train.py" $COMMON > "$OUT/plain.log" 2>&1 || exit $?
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
  "$ROOT/train.py" $COMMON > "$OUT/torchrun.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import json, sys, os
out = sys.argv[1]
import re
res = {}
for tag in ("plain", "torchrun"):
    txt = open(os.path.join(out, f"{tag}.log")).read()
    m = re.search(r"(\d+) steps in ([\d.]+)s \(([\d.]+) pairs/s\); steady state after (\d+) steps: ([\d.]+) pairs/s", txt)
    res[tag] = {"steps": int(m.group(1)), "pairs_per_s_all": float(m.group(3)),
                "steady_pairs_per_s": float(m.group(5)), "steady_from_step": int(m.group(4))} if m else {"error": txt[-500:]}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res))
PY
