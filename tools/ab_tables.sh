set -e
CFG=3 ROUNDS=3 VARIANTS="T1:--scene table;T2:--scene table --batch 2 --inflight 4;S1:--scene table-spec;S2:--scene table-spec --batch 2 --inflight 4" bash tools/ab_issue.sh
