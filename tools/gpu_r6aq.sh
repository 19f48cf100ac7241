set -e
O=gpurun_out/r6aq; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
bash tools/lib_ab_multi.sh $O/ab_cfg3.txt cfg3 variants/libgsrast_pz_end.so gaussian_splatting_lightning_amd/libgsrast.so
bash tools/lib_ab_multi.sh $O/ab_cfg5.txt cfg5 variants/libgsrast_pz_end.so gaussian_splatting_lightning_amd/libgsrast.so
bash tools/lib_ab_multi.sh $O/ab_cfg2.txt cfg2 variants/libgsrast_pz_end.so gaussian_splatting_lightning_amd/libgsrast.so
for i in 1 2; do
  GSR_LIB=variants/libgsrast_pz_end.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step > $O/prev_$i.json 2>&1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step > $O/new_$i.json 2>&1
done
