# round 6: residency slope of the throughput configs (verdict r05 item 4's premise): C3 / C4 at one GPU
# with the persistent grid capped -- fp32 (3 workgroups per CU resident: 768) at 512 / 768, fp64 (2 per
# CU: 512) at 384 / 512
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
OPTS="GRID=512|" bash tools/gpu_ab_opts.sh --dtype f32 --no-path --extras C3,C4_1gpu --extra-steps 4 | tee $O/r06j_grid_f32.log
OPTS="GRID=384|" bash tools/gpu_ab_opts.sh --dtype f64 --no-path --extras C3,C4_1gpu --extra-steps 4 | tee $O/r06j_grid_f64.log
echo ALLOK
