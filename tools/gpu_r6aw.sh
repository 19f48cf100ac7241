set -e
O=gpurun_out/r6aw; mkdir -p $O
B=gaussian_splatting_lightning_amd/libgsrast.so; V=variants/libgsrast_fwd_pf.so
bash tools/lib_ab_multi.sh $O/ab_cfg3.txt cfg3 $B $V $B $V
bash tools/lib_ab_multi.sh $O/ab_cfg5.txt cfg5 $B $V
bash tools/lib_ab_multi.sh $O/ab_cfg2.txt cfg2 $B $V
