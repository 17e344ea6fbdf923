# A/B runs + chained 32768^2 timelines in one call (bash tools/gpu_r3b.sh <tag>)
set -e
bash tools/gpu_ab_base.sh $1
bash tools/gpu_trace6.sh $1
