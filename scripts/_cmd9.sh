cd $GRAFT_REPO_ROOT
PYTEST_ARGS="" BENCH_ARGS="--steps 64 --warmup 4" bash scripts/gpu_check.sh || exit 1
TAG=r01_fused BENCH_ARGS="--steps 64 --warmup 4 --no-cpu-baseline" bash scripts/gpu_prof.sh || exit 1
TAG=r01_split BENCH_ARGS="--steps 64 --warmup 4 --no-cpu-baseline --split" bash scripts/gpu_prof.sh || exit 1
TAG=pmcf PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE|FETCH_SIZE|WRITE_SIZE|SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH SQ_INSTS_VALU_FP64" bash scripts/gpu_pmc.sh
