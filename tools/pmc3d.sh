# PMC passes over the 3D solve (tools/tune3d.py, one configuration), one
# rocprofv3 --pmc run each:  bash tools/pmc3d.sh <tag> <size> <sweep,rows,kc>
set -e
export TMPDIR=/tmp
tag=$1; n=$2; cfg=$3
out=gpurun_out/pmc3d_$tag
mkdir -p $out
T="python tools/tune3d.py --size $n --iters 20 --reps 1 --configs $cfg"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out -o trace --output-format csv -- $T > $out/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out -o fetch --output-format csv -- $T > $out/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out -o write --output-format csv -- $T > $out/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES -d $out -o sq --output-format csv -- $T > $out/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_SALU -d $out -o lds --output-format csv -- $T > $out/lds.log 2>&1
