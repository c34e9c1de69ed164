# Winograd instance sweep (SA_WINO_CFG) + ablation on the deep layers
for c in 0 1 2; do echo "cfg=$c"; SA_WINO_CFG=$c python tools/conv_f32_bench.py 3232 5 deep | sed 's/wgrad.*|//'; done
for a in 1 3; do echo "ablate=$a"; SA_WINO_ABLATE=$a python tools/conv_f32_bench.py 3232 5 "res32 18x24" | sed 's/wgrad.*|//'; done
