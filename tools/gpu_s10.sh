bash tools/gpu_session.sh \
 "curve|900|python -u tools/learning_curve.py --level synthetic_memory --torso deep --dtype fp32 --height 72 --width 96 --batch_size 32 --unroll_length 100 --num_actors 48 --frames 4000000 --log_every_frames 200000 --out gpurun_out/r3_learning_headline.jsonl"
