cd $GRAFT_REPO_ROOT
for mode in 0 1 2 4 7; do GDSP_DEBUG_COPY=$mode timeout -k 5 120 python scripts/debug_race.py || exit 1; done
TORCH_FIRST=1 timeout -k 5 120 python scripts/debug_race.py
