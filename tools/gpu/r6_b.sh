set -o pipefail
OUT=r6b bash tools/gpu/r6_groups.sh && OUT=r6b bash tools/gpu/r6_stage_ab.sh
