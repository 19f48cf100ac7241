set -e
export TMPDIR=/tmp
O=gpurun_out/r6ae; mkdir -p $O
R5=$PWD/variants/r5tree/gaussian_splatting_lightning_amd/libgsrast.so
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step > $O/B_$i.json 2>&1
  GSR_TUNE=xcd_lpt=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step > $O/X_$i.json 2>&1
  GSR_LIB=$R5 timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step > $O/C_$i.json 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p6 -o run -- python bench.py --no-cpu-baseline --no-train-step --steps 50 > $O/p6.log 2>&1
GSR_LIB=$R5 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p5 -o run -- python bench.py --no-cpu-baseline --no-train-step --steps 50 > $O/p5.log 2>&1
