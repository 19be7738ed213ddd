# Round 6: kvar with the stream-K W^T A arms (bit identity vs the engine's big tile, interleaved timings).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 300 ./tools/kvar 200 10 > $O/kvar.txt 2>&1; rc=$?
grep -E "stream-K|W\^T A|==|k_wta2|16 waves|items" $O/kvar.txt | head -60; exit $rc
