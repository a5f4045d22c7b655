#!/bin/bash
# Scratch GPU step (edited per experiment; inside gpurun): bash tools/scratch_gpu.sh
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
cat > /tmp/one.py <<'PY'
import sys, os
sys.path.insert(0, "diamond-types_amd"); sys.path.insert(0, "tests")
import dt_amd, golden_data as G
out = []
for name in ["friendsforever", "node_nodecc", "automerge-paper", "rustcode", "seph-blog1", "sveltecomponent"]:
    data = G.dt_bytes(name) if name in G.DT_FILES else dt_amd.apply_edits_push_merge(G.trace(name)["txns"]).encode()
    b = dt_amd.Batch(docs=[data], staging="device"); b.run(); b.sync()
    ts = sorted(b.run_timed() for _ in range(5))
    out.append(f"{name} {ts[2]:.2f}/{len(b.segments(0))}")
print("W", os.environ.get("DTGPU_SEG_W"), " ".join(out), flush=True)
PY
for w in 24 32 48 96 128 256; do
DTGPU_SEG_W=$w timeout -k 10 200 python -u /tmp/one.py || exit 1
done
for w in 64; do
DTGPU_SEG_W=$w timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done
