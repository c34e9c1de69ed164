for a in 0 1 2 4 8 6 3; do echo "ablate=$a"; SA_WINO_ABLATE=$a python tools/conv_f32_bench.py 3232 5 "res32 18x24" | sed 's/wgrad.*|//'; done
