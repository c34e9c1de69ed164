C="python -u tools/learning_curve.py --level synthetic_memory --torso deep --dtype fp32 --log_every_frames 200000 --out gpurun_out/curves.jsonl --height 72 --width 96 --batch_size 32 --unroll_length 100 --num_actors 48"
bash tools/gpu_session.sh \
 "ref|400|$C --frames 3000000 --learning_rate 0.00048 --entropy_cost 0.00025" \
 "torch|700|$C --frames 2000000 --learning_rate 0.0003 --backend torch"
