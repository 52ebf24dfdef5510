# Round 5, first GPU job: identity, scalar-gather A/B (k_rays_fxs at 65536 / 8192 cars, k_rays_fx at
# 8192 / 4096 / 2048), the previous commit's build, the learner tests, small-shard PMC, the bench.
set -o pipefail
bash scripts/gpu_run.sh r05a quick &&
AB_ENVS=65536,8192 AB_SIMT=1 AB_VARIANTS="sg0:REFILL=1,LANES=2,F110_FXS_SG=0;sg1:REFILL=1,LANES=2,F110_FXS_SG=1;sg2:REFILL=1,LANES=2,F110_FXS_SG=2" \
    bash scripts/gpu_run.sh r05a ab &&
AB_ENVS=8192,4096,2048 AB_SIMT=1 AB_VARIANTS="fx0:REFILL=0,LANES=1,F110_FX_SG=0;fx1:REFILL=0,LANES=1,F110_FX_SG=1;fx2:REFILL=0,LANES=1,F110_FX_SG=2" \
    bash scripts/gpu_run.sh r05b ab &&
AB_ENVS=65536,8192 AB_SIMT=1 AB_VARIANTS="head:REFILL=1,LANES=2" bash scripts/gpu_run.sh r05a abhead &&
AB_ENVS=8192,4096,2048 AB_SIMT=1 AB_VARIANTS="head:REFILL=0,LANES=1" bash scripts/gpu_run.sh r05b abhead &&
bash scripts/gpu_run.sh r05a bench learner dpgraph pmcsmall
