set -o pipefail
cd $GRAFT_REPO_ROOT/tools/microbench
for cfg in "0 8 1 16" "1 8 1 16" "2 8 1 16" "0 16 1 8" "1 16 1 8" "2 16 1 8" "1 4 1 16" "1 8 2 16" "0 8 2 16"; do
  timeout -k 5 60 ./mb_stream $cfg || exit 1
done
