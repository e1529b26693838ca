set -e
export TMPDIR=/tmp
for t in 32,8,0 16,16,0 64,4,0; do FAMG_XSCS_TILE=$t bash scripts/prof_c3.sh c3t > /dev/null; echo "== $t"; grep -E "xscs|per V-cycle" gpurun_out/c3t.txt | sed -n '1,5p'; done
for t in 32,8,0 16,16,0; do FAMG_XSCS_TILE=$t bash scripts/prof_c2.sh c2t > /dev/null; echo "== $t"; grep -E "xscs|per V-cycle" gpurun_out/c2t.txt | sed -n '1,7p'; done
