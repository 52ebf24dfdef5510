# Host-side sanitizer run (CPU only, this container): builds the host code of
# libf110.so (EDT, host tables, padded-table builder, beam runs, map cache,
# C ABI) and the C oracle with AddressSanitizer + UndefinedBehaviorSanitizer,
# then runs the CPU test suite against those builds.  Device code is built as
# usual (-Xarch_host puts the sanitizers on the host side only).
#
#   bash scripts/sanitize.sh            -> build/sanitize/{libf110.so,liboracle.so}, pytest -m "not gpu"
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/build/sanitize
mkdir -p "$OUT"
LLVM=/opt/rocm/lib/llvm
SAN="-fsanitize=address -fsanitize=undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"
C=$R/f110_gymnasium_ros2_jazzy_amd/csrc
HOSTSAN=""
for f in $SAN; do HOSTSAN="$HOSTSAN -Xarch_host $f"; done
/opt/rocm/bin/hipcc -O1 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
    -fvisibility=hidden -shared-libsan $HOSTSAN \
    $C/f110_kernels.hip $C/f110_opponent.hip $C/f110_reward.hip $C/f110_replay.hip $C/f110_adam.hip \
    $C/f110_ddpg.hip $C/f110_gemm.hip $C/f110_capi.cpp $C/f110_replay_capi.cpp -o "$OUT/libf110.so"
# the oracle with the same (clang) sanitizer runtime; OpenMP pragmas ignored (serial)
$LLVM/bin/clang -O1 -fPIC -std=c11 -ffp-contract=off -fno-fast-math -fno-builtin-sin -fno-builtin-cos \
    -fno-builtin-sincos -Wno-unknown-pragmas -D_GNU_SOURCE -shared -shared-libsan $SAN \
    "$R/oracle/f110_oracle.c" -o "$OUT/liboracle.so" -lm
RT=$($LLVM/bin/clang --print-file-name=libclang_rt.asan-x86_64.so)
cd "$R"
# python is not instrumented: the runtime is preloaded; leaks of the interpreter are not ours
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:verify_asan_link_order=0:log_path=$OUT/asan \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=$OUT/ubsan \
F110_LIB="$OUT/libf110.so" F110_ORACLE_LIB="$OUT/liboracle.so" \
    python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider "$@"
