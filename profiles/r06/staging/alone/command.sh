# q8_stage_kernel alone on an idle GPU (tools/stage_alone.py under rocprofv3 --kernel-trace --stats)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6sa}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o s --output-format csv -- python3 $R/tools/stage_alone.py > $O/run.log 2>&1
