set -e
O=gpurun_out/r6an; mkdir -p $O
for L in variants/libgsrast_pz_end.so variants/libgsrast_pz_start.so; do
  n=$(basename $L .so)
  for c in cfg3 cfg2; do
    GSR_LIB=$L timeout -k 10 300 python tools/stage_ab.py --config $c --knob bwd_prezero=1,0 --rounds 8 --steps 5 > $O/${n}_$c.txt 2>&1
  done
  GSR_LIB=$L timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob bwd_prezero=1,0 --rounds 4 --steps 3 > $O/${n}_cfg5.txt 2>&1
done
