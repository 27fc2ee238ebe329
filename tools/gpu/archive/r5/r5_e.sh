# r5: emit tile keys precomputed, lane-striped radix histogram; one-sweep tile size sweep on tri_find_mr RMAT-20
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_triangles.py tests/test_kernels_gpu.py tests/test_ooc_hot_key.py > $O/e_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/e_trimr20.txt 2>&1 &&
MRH_RX_KIT=16 timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/e_trimr20_k16.txt 2>&1 &&
MRH_RX_KIT=24 timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/e_trimr20_k24.txt 2>&1 &&
timeout -k 10 400 python -u tools/trimr_time.py 22 > $O/e_trimr22.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/etri -o run -- python -u tools/trimr_time.py 20 > $O/e_ptri.txt 2>&1
