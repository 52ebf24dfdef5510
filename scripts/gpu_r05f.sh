# Round 5: validation of the new size rules (k_rays_fxs everywhere): GPU suite, smoke, bench (default and
# the driver's settings), the 65536-car profile + PMC, small-shard PMC, C4 and C5 lines.
set -o pipefail
bash scripts/gpu_run.sh r05f suite smoke bench bench20 pmc pmcsmall c4 c4one c5
