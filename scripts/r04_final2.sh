#!/bin/bash
# Round-4 closing set at HEAD: scripts/r04_final.sh (GPU suite, smoke, bench
# line, 2-rank rehearsals) + rocprofv3 kernel stats of the c4 and c5 bench
# commands.  usage: scripts/r04_final2.sh TAG
set -o pipefail
TAG=${1:-r04x}
bash scripts/r04_final.sh $TAG || exit 1
bash scripts/prof_round.sh $TAG "c4 c5" "" || exit 1
