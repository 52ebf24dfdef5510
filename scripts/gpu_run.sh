# One parameterised GPU-box job (run through gpurun from the repo root):
#
#   bash scripts/gpu_run.sh TAG STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failure ends
# the job (no GPU step runs after a failed / faulted / timed-out one).  Output
# goes to gpurun_out/TAG/.  Steps:
#   suite      pytest -m gpu (one process, per-test timeout)
#   lgemm      tests/test_gpu_learner_gemm.py, scripts/learner_gemm_mb.py (+ its rocprofv3 kernel stats)
#   lgemmpmc   two PMC passes (SQ wait / MFMA busy; TA busy) over scripts/learner_gemm_mb.py
#   lgab       scripts/learner_gemm_mb.py once per alternate build ab_libs/*.so (F110_LIB)
#   learner    tests/test_gpu_replay.py + tests/test_gpu_ddpg_heads.py (the DDPG learner)
#   dpgraph    tests/test_gpu_dp_graphs.py (two gloo ranks on the GPU: step graphs vs eager)
#   c5prof     scripts/profile_c5.py TAG (C5 bench + rocprofv3 kernel stats by stage) -> gpurun_out/prof_c5_TAG/
#   quick      the dispatch-variant tests of tests/test_gpu_batch.py only
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py (defaults) -> bench.json
#   bench20    python bench.py --steps 20 --warmup 5 (the driver's settings) -> bench20.json
#   prof       rocprofv3 --kernel-trace --stats over bench.py (no cpu leg) -> prof/, kernel_stats.csv
#   pmc        scripts/profile_round.py TAG (kernel trace + PMC passes of the headline ray kernel)
#   ab         scripts/ray_ab.py with the caller's AB_* environment -> ab.json
#   abhead     the same A/B with ab_libs/head.so (F110_LIB: the previous commit's build) -> abhead.json
#   libab      scripts/lib_ab.py: this build against ab_libs/head.so in one process (65536 / 8192 cars) -> libab.json
#   libab2     the same for 8192 two-agent envs -> libab2.json
#   c4s / c5s  bench.py C4 / C5 at the driver's --steps 20 --warmup 5 -> c4s.json / c5s.json
#   rules      scripts/shard_rules.py with the caller's SR_* environment -> rules.jsonl
#   pmcsmall   PMC passes (no kernel trace) at 8192 and 4096 cars, the default ray kernel and k_rays_fxs
#   trace      scripts/wave_trace.py (WT_ENVS), one context and bench's sub-shards -> trace_*.json
#   agents     scripts/agents_probe.py (k_agents per launch: car counts, RK4 / Euler) -> agents.json
#   post       scripts/post_probe.py (k_post_multi per launch at 4096 / 8192 two-agent envs) -> post.json
#   c4one      bench.py --agents 2 --global-envs 8192 --runner one (one context) -> c4one.json
#   x2         the headline bench as 2 ranks on the one GPU over gloo, self-launched by bench.py --gpus 2
#   handoff    tests/test_gpu_handoff.py (the two-agent hand-off mask's hard cases)
#   weak       C3's weak-scaling shape: 2 ranks x 8192 envs per GPU on the one GPU (gloo) and 1 rank x 16384
#              envs, same K / W / seed: their trajectory_digest must agree
#   c5x2       the DDPG bench as 2 ranks on the one GPU over gloo (the data-parallel path, no step graphs)
#   c4 / c5    bench.py --agents 2 --global-envs 8192 / --workload ddpg -> c4.json / c5.json
set -o pipefail
TAG=${1:?tag}
shift
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
run() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    if [ $rc -ne 0 ]; then
        echo "step $name failed rc=$rc" >&2
        tail -30 "$OUT/$name.err" >&2
        tail -30 "$OUT/$name.out" >&2
        exit $rc
    fi
}
for step in "$@"; do
    case $step in
        suite) run suite 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
        quick) run quick 600 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -v --timeout 300 --timeout-method thread \
                   -p no:cacheprovider -k "step_n or simt or refill_kernel" ;;
        lgemm) run lgemm 600 python -u -m pytest tests/test_gpu_learner_gemm.py -m gpu -x -v --timeout 120 \
                   --timeout-method thread -p no:cacheprovider &&
               run lgemm_mb 300 python -u scripts/learner_gemm_mb.py && cp "$OUT/lgemm_mb.out" "$OUT/lgemm_mb.json" &&
               run lgemm_prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/lgemm_prof" -o run -- \
                   python3 scripts/learner_gemm_mb.py ;;
        lgemmpmc) run lgemm_pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
                      SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
                      -d "$OUT/lgemm_pmc1" -o run -- python3 scripts/learner_gemm_mb.py &&
                  run lgemm_pmc2 120 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum SQ_INSTS_VMEM_RD \
                      GRBM_GUI_ACTIVE --output-format csv -d "$OUT/lgemm_pmc2" -o run -- \
                      python3 scripts/learner_gemm_mb.py ;;
        learner) run learner 600 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_ddpg_heads.py -m gpu -x -v \
                     --timeout 200 --timeout-method thread -p no:cacheprovider ;;
        lgab) for lib in ab_libs/*.so; do  # the microbench per alternate build (F110_LIB)
                  n=$(basename "$lib" .so)
                  F110_LIB=$R/$lib run "lgab_$n" 300 python -u scripts/learner_gemm_mb.py || exit $?
              done ;;
        dpgraph) run dpgraph 600 python -u -m pytest tests/test_gpu_dp_graphs.py -m gpu -x -v --timeout 400 \
                     --timeout-method thread -p no:cacheprovider ;;
        c5prof) run c5prof 900 python -u scripts/profile_c5.py "$TAG" ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python -u bench.py && cp "$OUT/bench.out" "$OUT/bench.json" ;;
        bench20) run bench20 600 python -u bench.py --steps 20 --warmup 5 && cp "$OUT/bench20.out" "$OUT/bench20.json" ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --steps 300 \
                  --no-cpu-baseline --no-secondary --no-full-outputs &&
              find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$OUT/kernel_stats.csv" ;;
        pmc) run pmc 900 python -u scripts/profile_round.py "$TAG" ;;
        ab) run ab 900 python -u scripts/ray_ab.py && cp "$OUT/ab.out" "$OUT/ab.json" ;;
        libab) run libab 900 python -u scripts/lib_ab.py && cp "$OUT/libab.out" "$OUT/libab.json" ;;
        libab2) AB_AGENTS=2 AB_ENVS=8192 run libab2 900 python -u scripts/lib_ab.py && cp "$OUT/libab2.out" "$OUT/libab2.json" ;;
        c4s) run c4s 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline --no-secondary --steps 20 \
                 --warmup 5 && cp "$OUT/c4s.out" "$OUT/c4s.json" ;;
        c5s) run c5s 600 python -u bench.py --workload ddpg --steps 20 --warmup 5 && cp "$OUT/c5s.out" "$OUT/c5s.json" ;;
        abhead) F110_LIB=$R/ab_libs/head.so run abhead 900 python -u scripts/ray_ab.py &&
                cp "$OUT/abhead.out" "$OUT/abhead.json" ;;
        rules) run rules 900 python -u scripts/shard_rules.py && cp "$OUT/rules.out" "$OUT/rules.jsonl" ;;
        pmcsmall) for e in 8192 4096; do  # the default dispatch (k_rays_fxs, 3 waves per car) and round 4's k_rays_fx
                      PROFILE_NO_TRACE=1 PROFILE_ENVS=$e run "pmc_$e" 600 python -u scripts/profile_round.py "$TAG" &&
                      PROFILE_NO_TRACE=1 PROFILE_ENVS=$e PROFILE_REFILL=0 run "pmc_${e}_fx" 600 \
                          python -u scripts/profile_round.py "$TAG" || exit $?
                  done ;;
        trace) WT_MODE=one run trace 600 python -u scripts/wave_trace.py && cp "$OUT/trace.out" "$OUT/trace_one.json" &&
               WT_MODE=shards run trace_shards 600 python -u scripts/wave_trace.py &&
               cp "$OUT/trace_shards.out" "$OUT/trace_shards.json" ;;
        c4) run c4 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline --no-secondary &&
            cp "$OUT/c4.out" "$OUT/c4.json" ;;
        agents) run agents 300 python -u scripts/agents_probe.py && cp "$OUT/agents.out" "$OUT/agents.json" ;;
        post) run post 300 python -u scripts/post_probe.py && cp "$OUT/post.out" "$OUT/post.json" ;;
        c4one) run c4one 600 python -u bench.py --agents 2 --global-envs 8192 --no-cpu-baseline --no-secondary \
                   --runner one && cp "$OUT/c4one.out" "$OUT/c4one.json" ;;
        x2) F110_SAME_DEVICE=1 F110_DIST_BACKEND=gloo run x2 600 python -u bench.py --gpus 2 --steps 20 \
                --warmup 5 && cp "$OUT/x2.out" "$OUT/x2.json" ;;
        handoff) run handoff 600 python -u -m pytest tests/test_gpu_handoff.py -m gpu -x -v --timeout 300 \
                     --timeout-method thread -p no:cacheprovider ;;
        weak) F110_SAME_DEVICE=1 F110_DIST_BACKEND=gloo run weak2 600 python -m torch.distributed.run --nnodes=1 \
                  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --envs-per-gpu 8192 \
                  --steps 20 --warmup 5 && cp "$OUT/weak2.out" "$OUT/weak2.json" &&
              run weak1 600 python -u bench.py --global-envs 16384 --steps 20 --warmup 5 --no-cpu-baseline \
                  --no-secondary && cp "$OUT/weak1.out" "$OUT/weak1.json" ;;
        c5x2) F110_SAME_DEVICE=1 F110_DIST_BACKEND=gloo run c5x2 600 python -u bench.py --gpus 2 --workload ddpg \
                  --steps 50 --warmup 20 && cp "$OUT/c5x2.out" "$OUT/c5x2.json" ;;
        c5) run c5 600 python -u bench.py --workload ddpg --steps 200 --warmup 20 && cp "$OUT/c5.out" "$OUT/c5.json" ;;
        *) echo "unknown step $step" >&2; exit 2 ;;
    esac
done
echo "[$(date +%T)] done" >&2
