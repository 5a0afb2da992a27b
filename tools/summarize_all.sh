#!/bin/bash
# Summarise a tools/profile_all.sh run (here, after gpurun merged it back) into
# profiles/<TAG>_{cfgN,table,tablespec}_*, with each configuration's PMC settings
# (kind, config, steps, frames per launch) as profile_all.sh ran them.
#   tools/summarize_all.sh gpurun_out/prof12 r06
set -e
SRC=${1:?source prefix}; TAG=${2:?tag}
run() { PROF_KIND=$1 PROF_CFG=$2 PROF_STEPS=$3 PROF_BATCH=$4 python3 tools/summarize_profiles.py "$5" "$6" "$7"; }
run pixel 3 20 1 "${SRC}_cfg3" "${TAG}_cfg3" cfg3
run pixel 4 20 1 "${SRC}_cfg4" "${TAG}_cfg4" cfg4
run pixel 5 20 1 "${SRC}_cfg5" "${TAG}_cfg5" cfg5
run pixel 2 120 20 "${SRC}_cfg2" "${TAG}_cfg2" cfg2
run pixel 1 120 20 "${SRC}_cfg1" "${TAG}_cfg1" cfg1
run table 3 20 2 "${SRC}_table" "${TAG}_table" cfg3
run table-spec 3 20 2 "${SRC}_tablespec" "${TAG}_tablespec" cfg3-spec
