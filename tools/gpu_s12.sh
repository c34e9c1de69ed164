C="python -u tools/learning_curve.py --level synthetic_memory --torso deep --dtype fp32 --log_every_frames 200000 --out gpurun_out/curves.jsonl --height 72 --width 96 --batch_size 32 --unroll_length 100 --num_actors 48 --frames 3000000"
bash tools/gpu_session.sh \
 "l3|400|$C --learning_rate 0.0003" \
 "l15|400|$C --learning_rate 0.00015" \
 "e1|400|$C --entropy_cost 0.01"
