#!/bin/bash
# Per-phase workgroup time of the one-kernel round at several slot counts.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for S in ${SLOTS:-256 512 1024 3000}; do
  GS_PHASE_PROFILE=1 timeout -k 10 120 python bench.py --no-cpu-baseline --slots "$S" --steps 60 --warmup 20 \
    > "gpurun_out/phase_$S.log" 2>&1 || { echo "slots=$S failed rc=$?"; tail -5 "gpurun_out/phase_$S.log"; exit 1; }
  python3 - "$S" <<'PY'
import json, sys
S = int(sys.argv[1])
d = json.loads(open(f"gpurun_out/phase_{S}.log").read().strip().splitlines()[-1])
ph = d.get("phases_wg_ms", {})
n = S * d["steps"]
print(f"slots={S} ms/step={d['ms_per_step']:.3f} edges/s={d['value']:.3e} per-WG-round us:",
      {k: (round(v * 1e3 / n, 1) if not (k.startswith("bfs_levels") or k.endswith("_cyc")) else v) for k, v in ph.items()})
PY
done
