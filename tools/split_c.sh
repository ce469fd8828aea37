set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
  for m in 0 1024 512; do
    GSR_SPLIT=$m timeout -k 10 300 python tools/graph_probe.py --configs C --steps 200 --rounds 1 --graph-only 2>&1 | grep graph | sed "s/^/split $m: /"
  done
done
