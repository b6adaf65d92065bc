# The driver's round-end GPU tiers in miniature: build check import, smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
