# Round 6: same-box A/B of the verify's wide-phase change (arm prewide = eee1ae5's library, new = this tree), 3
# alternating reps, the 1M headline (424 of 640 slots take the wide phase) and the 500k shard through the exchange.
set -o pipefail
R=$GRAFT_REPO_ROOT
REPS=3 bash $R/tools/gpu/r6_ab.sh r6abw/h1m "--steps 20 --warmup 5 --steady-steps 1000" "prewide:" "new:" &&
REPS=2 bash $R/tools/gpu/r6_ab.sh r6abw/x500k "--steps 20 --warmup 5 --steady-steps 1000 --docs 500000 --exchange-1rank" "prewide:" "new:"
