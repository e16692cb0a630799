set -uo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/mgx_debug.py sf3d_edit 2>&1 | tail -20
timeout -k 10 200 python -u tools/mgx_debug.py nb_xt 2>&1 | tail -12
