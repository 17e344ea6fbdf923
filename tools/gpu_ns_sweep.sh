export TMPDIR=/tmp
o=gpurun_out/ns_sweep_$1.txt; : > $o
for r in 2 4 8; do for b in 1024 2048 4096; do
  echo "rows $r blocks $b" >> $o
  MISOR_ADAPT_ROWS=$r MISOR_RED_BLOCKS=$b timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/nss_$r$b -o t --output-format csv -- python bench.py --workload ns --no-cpu-baseline --steps 6 --warmup 2 > /dev/null 2>&1 || exit 1
  grep -h "adapt_absmax\|fg_rhs" gpurun_out/nss_$r$b/t_kernel_stats.csv | cut -d, -f1,4 | sed 's/(.*"//' >> $o
done; done
