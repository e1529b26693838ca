set -e
export TMPDIR=/tmp
cat > /tmp/ac.py <<'PY'
import os, sys
import torch
torch.zeros(1, device="cuda:0")
sys.argv = ["x", os.environ.get("BUILDS", "4"), "0"]
sys.path[:0] = ["faer-amg_amd", "oracle"]
import faer_amg_amd as fa
fa.set_alloc_policy(int(os.environ.get("POLICY", "1")))
src = open("scripts/alloc_coherence.py").read().replace("dims = (64, 64, 64)", "dims = (%s,)" % os.environ.get("DIMS", "64, 64, 64"))
exec(src)
PY
echo "== 128^3 contiguous"; DIMS="128, 128, 128" FAMG_ALLOC_DEBUG=1 FAMG_ALLOC_EXPERIMENT=1 FAMG_CHECK_STORAGE=1 timeout -k 10 400 python /tmp/ac.py > gpurun_out/ac1.log 2>&1 || true; echo "contiguous allocs: $(grep -c 'alloc contiguous' gpurun_out/ac1.log)"; grep -E "^build|mismatch|Error" gpurun_out/ac1.log | head -6
