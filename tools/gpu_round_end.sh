#!/bin/bash
# Everything the round end needs from one GPU box: the whole -m gpu suite, the default bench line
# and its kernel trace (tools/gpu_full.sh), both training steps' kernel traces, and the final tree's
# PMC passes + kernel stats (tools/gpu_pmc_final.sh).  Usage (GPU box): bash tools/gpu_round_end.sh <tag>
set -u
TAG=$1
bash tools/gpu_full.sh $TAG || exit 1
bash tools/gpu_train_trace.sh $TAG || exit 1
bash tools/gpu_pmc_final.sh $TAG || exit 1
echo ROUND_END_DONE
