# Replay-sampling A/B on the GPU box: scripts/replay_probe.py (1M-row buffer, C5's shapes) once per
# build in RPAB_LIBS (names under ab_libs/, "tree" = the in-tree libf110.so), twice each
# interleaved, then one rocprofv3 kernel trace per build, then tests/test_gpu_replay.py.
#   bash scripts/gpu_rpab.sh TAG
set -o pipefail
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
LIBS=${RPAB_LIBS:-"head tree"}
use() { if [ "$1" = tree ]; then unset F110_LIB; else export F110_LIB=$R/ab_libs/$1.so; fi; }
for rep in 1 2; do
  for lib in $LIBS; do
    use $lib
    RP_FILL=1048576 RP_STEPS=300 timeout -k 10 200 python -u scripts/replay_probe.py >> $O/probe_$lib.jsonl 2>> $O/err.txt || exit 1
  done
done
for lib in $LIBS; do
  use $lib
  RP_FILL=1048576 RP_STEPS=300 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$lib -o run -- \
      python3 scripts/replay_probe.py > $O/prof_$lib.out 2>&1 || exit 1
done
unset F110_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > $O/tests.out 2>&1
