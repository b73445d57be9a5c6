cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/c5_long.sh r05d 3500 "GPC_NO_EXTENSIONS=1" 2>&1 | tail -5
