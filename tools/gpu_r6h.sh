# Round 6: the stream-K whole-round order as an L2-residency / DVFS probe: kvar timings of both
# orders (bit identity included), then FETCH_SIZE / WRITE_SIZE passes with GRBM_GUI_ACTIVE (clock) of kvar's pmc mode.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 300 ./tools/kvar 200 10 > $O/kvar.txt 2>&1 || exit 1
grep -E "stream-K|16 waves, GREG \(engine\)" $O/kvar.txt | head -30
timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- ./tools/kvar 200 3 pmc > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-include-regex "k_wta2" --output-format csv -d $O/FETCH_SIZE -o run -- ./tools/kvar 200 3 pmc > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-include-regex "k_wta2" --output-format csv -d $O/WRITE_SIZE -o run -- ./tools/kvar 200 3 pmc > $O/write.log 2>&1 || exit 1
python3 tools/sk_order_pmc.py $O 3
