# interleaved A/B of the single-rank loop test: two levels (MISOR_FINISH2=1, default) vs one kernel (0)
set -e
export TMPDIR=/tmp
o=gpurun_out/fin2; mkdir -p $o
for f in 1 0 1 0 1 0; do
  MISOR_FINISH2=$f timeout -k 10 200 python bench.py --steps 140 --warmup 7 --no-cpu-baseline >> $o/finish2_$f.json 2>>$o/err.log
done
