set -e
export TMPDIR=/tmp
for w in 64 40; do FAMG_BSR_MAXW=$w bash scripts/prof_c5.sh c5w$w > /dev/null; echo "== maxw $w"; sed -n '/per launch/,$p' gpurun_out/c5w$w.txt | head -20; grep -o '"value": [0-9.]*' gpurun_out/c5w$w.log | head -1; done
