#!/bin/bash
# The round's profile set (tools/profile_round.sh) for every BASELINE config and
# the scene-table kernels, each with the frames per launch bench.py times.
set -e
R=${1:-gpurun_out/prof6}
PROF_KIND=pixel PROF_CFG=3 PROF_STEPS=20 PROF_BATCH=1 bash tools/profile_round.sh $R"_cfg3" --steps 20 --warmup 5
PROF_KIND=pixel PROF_CFG=4 PROF_STEPS=20 PROF_BATCH=1 bash tools/profile_round.sh $R"_cfg4" --config 4 --steps 20 --warmup 5
PROF_KIND=pixel PROF_CFG=5 PROF_STEPS=20 PROF_BATCH=1 bash tools/profile_round.sh $R"_cfg5" --config 5 --steps 20 --warmup 5
PROF_KIND=pixel PROF_CFG=2 PROF_STEPS=120 PROF_BATCH=20 bash tools/profile_round.sh $R"_cfg2" --config 2 --steps 120 --warmup 5
PROF_KIND=pixel PROF_CFG=1 PROF_STEPS=120 PROF_BATCH=20 bash tools/profile_round.sh $R"_cfg1" --config 1 --steps 120 --warmup 5
PROF_KIND=table PROF_CFG=3 PROF_STEPS=20 PROF_BATCH=2 bash tools/profile_round.sh $R"_table" --scene table --steps 20 --warmup 5
PROF_KIND=table-spec PROF_CFG=3 PROF_STEPS=20 PROF_BATCH=2 bash tools/profile_round.sh $R"_tablespec" --scene table-spec --steps 20 --warmup 5
echo all-done
