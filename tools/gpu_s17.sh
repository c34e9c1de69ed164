E="FRAMES=6144000 bash tools/e2e_actors.sh"
bash tools/gpu_session.sh \
 "s3|280|$E s3 96 2 --inference_server=true --actor_group_splits=3" \
 "s4|280|$E s4 96 2 --inference_server=true --actor_group_splits=4" \
 "g4|280|$E g4 96 4 --inference_server=true" \
 "g3s3|280|$E g3s3 96 3 --inference_server=true --actor_group_splits=3" \
 "g1|280|$E g1b 96 1 --inference_server=true"
