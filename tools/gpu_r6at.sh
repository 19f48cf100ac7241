set -e
O=gpurun_out/r6at; mkdir -p $O
bash tools/lib_ab_multi.sh $O/ab_cfg3.txt cfg3 gaussian_splatting_lightning_amd/libgsrast.so variants/libgsrast_zf_plain.so
bash tools/lib_ab_multi.sh $O/ab_cfg5.txt cfg5 gaussian_splatting_lightning_amd/libgsrast.so variants/libgsrast_zf_plain.so
