set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6tl; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/x125 -o t -- python3 $R/tools/step_timeline.py run --docs 125000 --x --restage > $O/x125.run 2>&1 &&
python3 $R/tools/step_timeline.py analyse $O/x125 > $O/x125.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/n125 -o t -- python3 $R/tools/step_timeline.py run --docs 125000 --restage > $O/n125.run 2>&1 &&
python3 $R/tools/step_timeline.py analyse $O/n125 > $O/n125.txt 2>&1
