#!/bin/bash
# A/B session on the GPU box: kernel time (one frame at a time) and bench wall time
# (frames in flight) of librm.so against tools/variants/librm_*.so, plus an optional
# parity check of each variant.  Usage: tools/ab_job.sh [cfg] [parity]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFG=${1:-3}
if [ "$2" = "parity" ]; then
  for so in tools/variants/librm_*.so; do
    RM_LIBRM=$so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread > gpurun_out/ab_parity_$(basename $so .so).log 2>&1 \
      || { echo "parity FAILED $so"; tail -20 gpurun_out/ab_parity_$(basename $so .so).log; exit 1; }
    echo "parity ok $so: $(tail -1 gpurun_out/ab_parity_$(basename $so .so).log)"
  done
fi
timeout -k 10 600 python -u tools/ab_kernel.py --cfg $CFG --rounds ${ROUNDS:-3} --frames 20 || exit 1
[ "${BENCH:-1}" = 0 ] && exit 0
for r in 1 2 3; do
  for so in opengl-raymarching-in-compute-shader_amd/librm.so tools/variants/librm_*.so; do
    RM_LIBRM=$so timeout -k 10 120 python bench.py --no-cpu-baseline --config $CFG --steps 60 --warmup 5 > /tmp/ab.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('/tmp/ab.json'));print('$(basename $so)', 'bench ms', d['ms_per_step'], 'fps', d['fps'])"
  done
done
