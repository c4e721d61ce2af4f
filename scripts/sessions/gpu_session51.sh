set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./scripts/ubench/issue_rmw
