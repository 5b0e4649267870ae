V=$GRAFT_REPO_ROOT/gnn-elasticity-predictor_amd/alignn_mi355x/variants
timeout -k 10 200 python tools/tconv_bench.py > gpurun_out/tb_base.log 2>&1 || exit 1
for v in noacc wpe2 pf2; do ALIGNN_HIP_LIB=$V/libalignn_hip_$v.so timeout -k 10 200 python tools/tconv_bench.py > gpurun_out/tb_$v.log 2>&1 || exit 1; done
for v in base noacc wpe2 pf2; do echo "== $v"; grep -v amdgpu gpurun_out/tb_$v.log; done
