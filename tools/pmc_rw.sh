set -euo pipefail
cd $GRAFT_REPO_ROOT
cp tools/ab/lib_nosb.so lssurf_amd/liblsqsurf.so
bash tools/pmc_normal.sh pmc_rw_nosb
python3 tools/pmc_summary.py gpurun_out/pmc_rw_nosb > gpurun_out/pmc_rw_nosb/summary.txt 2>&1 || true
cat gpurun_out/pmc_rw_nosb/summary.txt | head -60
