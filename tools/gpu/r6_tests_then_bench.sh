# GPU box: a few GPU test files, then the full 1-GPU bench; stops after a
# crash or time limit (pytest rc 0/1 = tests ran, anything else = stop)
set -u
out=gpurun_out/$1; shift
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu "$@" > "$out/tests.log" 2>&1
rc=$?
echo "tests rc=$rc" >> "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py --detail-out "$out/bench_detail.json" > "$out/bench.out" 2> "$out/bench.err"
