set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L="4099 4507 5003 5449 4106 4253"
for r in 1 2; do
timeout -k 10 300 python scripts/dev/parts13_ab.py $L > gpurun_out/p13_off_$r.jsonl 2>&1 || { tail gpurun_out/p13_off_$r.jsonl; exit 1; }
GDSP_BLU_PARTS13=1 timeout -k 10 300 python scripts/dev/parts13_ab.py $L > gpurun_out/p13_on_$r.jsonl 2>&1 || { tail gpurun_out/p13_on_$r.jsonl; exit 1; }
done
for f in gpurun_out/p13_*.jsonl; do echo $f; python -c "import sys,json;[print(d['n'],d['m'],d['parts'],d['ms'],'%.1e'%d['err']) for d in map(json.loads,[l for l in open('$f') if l.startswith('{')])]"; done
