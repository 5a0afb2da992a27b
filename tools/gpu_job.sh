#!/bin/bash
# One GPU-box session (gpurun): the -m gpu suite, the default bench line and the
# round's profile set.  Every GPU step has its own time limit; steps chain with &&.
#   tools/gpu_job.sh TAG [tests|bench|prof ...]   (default: all three)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}; shift
STEPS=${STEPS:-all}
[ $# -gt 0 ] && STEPS="$*"
mkdir -p gpurun_out
run() { case " $STEPS " in *" $1 "*|" all ") return 0;; *) return 1;; esac; }
ok=0
if run tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
if run bench; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json \
    2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_bench.json
fi
if run prof; then
  PROF_STEPS=20 timeout -k 10 900 bash tools/profile_round.sh gpurun_out/prof_${TAG} --steps 20 --warmup 5 \
    || { echo "profile failed"; exit 1; }
  # summarise here afterwards: PROF_STEPS=20 python tools/summarize_profiles.py gpurun_out/prof_TAG TAG cfg3
fi
exit $ok
