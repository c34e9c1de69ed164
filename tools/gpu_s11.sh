C="python -u tools/learning_curve.py --level synthetic_memory --torso deep --dtype fp32 --log_every_frames 200000 --out gpurun_out/curves.jsonl"
bash tools/gpu_session.sh \
 "a|400|$C --height 72 --width 96 --batch_size 8 --unroll_length 20 --num_actors 16 --frames 1200000" \
 "b|400|$C --height 36 --width 48 --batch_size 32 --unroll_length 100 --num_actors 48 --frames 4000000" \
 "c|600|$C --backend torch --height 72 --width 96 --batch_size 32 --unroll_length 100 --num_actors 48 --frames 2000000"
