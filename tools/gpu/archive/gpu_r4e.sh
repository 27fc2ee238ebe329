# r4: with_file_io breakdown probe + PageRank setup stages
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/ii_fileio_probe.py > $O/fileio_probe.log 2>&1 &&
bash tools/pr_setup_stages.sh
