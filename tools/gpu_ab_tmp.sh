set -o pipefail
cd "$GRAFT_REPO_ROOT"
ROUNDS=5 bash tools/ab_job.sh 3 parity || exit 1
for c in 1 2 4 5; do timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r02_cfg$c.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('gpurun_out/r02_cfg$c.json'));print('cfg$c', d['ms_per_step'], d['fps'], d['value'], d['parity'], d['roofline']['frac'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"; done
