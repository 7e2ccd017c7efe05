# RCCL settings against the closing device sync's cost on RCCL's own streams (window_cost at 125k, 1-rank exchange).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5renv}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/window_cost.py 125000 --x > $O/default.txt 2>&1 &&
NCCL_GRAPH_MIXING_SUPPORT=0 timeout -k 10 200 python3 $R/tools/window_cost.py 125000 --x > $O/graph_mixing_0.txt 2>&1 &&
NCCL_LAUNCH_ORDER_IMPLICIT=1 timeout -k 10 200 python3 $R/tools/window_cost.py 125000 --x > $O/launch_order_implicit_1.txt 2>&1
