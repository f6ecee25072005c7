# Per-dispatch kernel trace of one mp_ilqr_solve at configs[2] (tools/ilqr_time.py --solve-only);
# analyse with: python tools/ilqr_iters.py gpurun_out/ilqr_tr/tr_kernel_trace.csv
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ilqr_tr -o tr -- python3 tools/ilqr_time.py --solve-only > gpurun_out/ilqr_tr.log 2>&1
grep solve gpurun_out/ilqr_tr.log
