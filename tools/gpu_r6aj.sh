set -e
O=gpurun_out/r6aj; mkdir -p $O
B=variants/libgsrast_base.so; Q1=variants/libgsrast_bwdq1.so; Q2=variants/libgsrast_bwdq2.so
Q3=variants/libgsrast_bwdq3.so
bash tools/lib_ab_multi.sh $O/ab_cfg3.txt cfg3 $B $Q1 $Q2 $Q3 $B $Q3
bash tools/lib_ab_multi.sh $O/ab_cfg5.txt cfg5 $B $Q1 $Q3
GSR_LIB=$Q1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "composite_variants or segmented or oracle or golden or reference or saturated" > $O/parity_q1.log 2>&1
