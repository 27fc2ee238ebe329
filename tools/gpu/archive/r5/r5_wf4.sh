# r5: 2-rank wordfreq shuffle on the device engine + the wordfreq extras of the record at 8 GiB
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_distributed_gpu.py tests/test_rccl_gpu.py -k "wordfreq or inverted or collate or rccl" > $O/wf4_tests.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --trifind-mr-scale 0 --file-io-steps 0 --dist-extras 0 > $O/wf4_bench.json 2> $O/wf4_bench.err
