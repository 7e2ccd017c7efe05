# Per-workgroup phases of one screen launch (tools/probe_screen, built in-tree as tools/probe_screen_r6): 125k and 500k
# rows, one and two int8 query pieces, the product's grids (224 beside a verify, 256 alone) and chunk sizes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6p}; mkdir -p $O; cd /tmp
P=$R/tools/probe_screen_r6
for a in "125000 224 2 0 1 0 2" "125000 224 2 0 1 0 1" "125000 256 2 0 1 0 2" "500000 224 4 0 1 0 1" "500000 256 4 0 1 0 1" "1000000 256 4 0 1 0 1"; do
  timeout -k 5 60 $P $a >> $O/probe.jsonl || exit 1
done
