#!/bin/bash
# Host AddressSanitizer run of the native engine (SURVEY.md §5 "race
# detection / sanitizers"; GPU ASan is not available on this pool).
#
# Rebuilds every host source (engine, C API, OINK) with -fsanitize=address
# into build/asan/libmrhip.so, linked with the normal gfx950 kernel objects,
# then runs on the CPU engine:
#   * tests/capi/capi_test.c  (every MR_* op family, multi-block reduce, ...)
#   * examples/c/cwordfreq.c as a 2-rank job over the store transport
#   * the oink executable on examples/oink/in.tri and in.cc
# Usage: bash tools/asan_check.sh   (after a normal build; ~3 min on 8 CPUs)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/asan
mkdir -p "$OUT/obj"
cd "$ROOT"
PYINC=$(python -c "from torch.utils.cpp_extension import include_paths; print(' '.join('-I'+p for p in include_paths()))")
TLIB=$(python -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
ABI=$(python -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
FLAGS="-O1 -g -std=c++17 -fPIC -fsanitize=address -fno-omit-frame-pointer -Wno-unused-result -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI=$ABI -I csrc -I /opt/rocm/include $PYINC"
SRCS=$(ls csrc/engine/*.cpp csrc/capi/*.cpp csrc/oink/*.cpp | grep -v -e bind.cpp -e oink/main.cpp)
echo "compiling $(echo $SRCS | wc -w) host sources with ASan"
printf '%s\n' $SRCS | xargs -P "${MAX_JOBS:-8}" -I{} sh -c 'o='"$OUT"'/obj/$(echo {} | tr / _).o; g++ '"$FLAGS"' -c {} -o $o'
LIBS="-L/opt/rocm/lib -L$TLIB -lamdhip64 -lc10_hip -ltorch_hip -lc10 -ltorch -ltorch_cpu -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib -Wl,-rpath,$TLIB"
g++ -shared -fsanitize=address -o "$OUT/libmrhip.so" "$OUT"/obj/*.o build/kernels/*.o $LIBS
gcc -g -fsanitize=address tests/capi/capi_test.c -I csrc/capi -L "$OUT" -lmrhip -Wl,-rpath,"$OUT" -o "$OUT/capi_test"
gcc -g -fsanitize=address examples/c/cwordfreq.c -I csrc/capi -L "$OUT" -lmrhip -Wl,-rpath,"$OUT" -o "$OUT/cwordfreq"
g++ $FLAGS csrc/oink/main.cpp -o "$OUT/oink" -L "$OUT" -lmrhip -Wl,-rpath,"$OUT" $LIBS

export HIP_VISIBLE_DEVICES= ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
W=$(mktemp -d)
echo "== capi_test"
"$OUT/capi_test" "$W" | tail -n 1
echo "== cwordfreq, 2 ranks"
mkdir -p "$W/docs"
for i in 0 1 2; do python -c "import random; random.seed($i); print(' '.join(random.choice(['aa','b','ccc','dd']) for _ in range(3000)))" > "$W/docs/f$i.txt"; done
PORT=$((20000 + RANDOM % 20000))
for r in 0 1; do
  WORLD_SIZE=2 RANK=$r LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT "$OUT/cwordfreq" -n 2 "$W/docs" > "$W/wf$r.txt" &
done
wait
cat "$W/wf0.txt"
for s in in.tri in.cc; do
  echo "== oink $s"
  (cd "$W" && "$OUT/oink" -in "$ROOT/examples/oink/$s" -var scale 8 | grep -E "Tri_find|CC_find")
done
rm -rf "$W"
echo "ASAN CLEAN"
