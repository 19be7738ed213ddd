# Round 6: the k_hupdate split-K combine arm -- NMFC_WTA_LASTSUM=1: k_wta2_sk's last-arriving
# chunk of every tile sums the tile's chunk partials (k_hupdate's order) so k_hupdate reads one.  Bit identity, an
# interleaved A/B of the C3 line, and FETCH/WRITE PMC passes of both arms.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "stream_k" --timeout 240 --timeout-method thread > $O/sk_tests.log 2>&1; rc=$?
tail -2 $O/sk_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for LS in 0 1; do
  NMFC_WTA_LASTSUM=$LS timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/ls${LS}_$rep.json 2> $O/ls${LS}_$rep.err || exit 1
  python3 -c "import json;d=json.load(open('$O/ls${LS}_$rep.json'));k=d['roofline']['kernels'];print('LASTSUM=$LS rep $rep', round(d['value'],2), 'wta', round(k['wta']['avg_ms'],4), 'hupd', round(k['hupdate']['avg_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done; done
for LS in 0 1; do for pass in FETCH_SIZE WRITE_SIZE; do
  NMFC_WTA_LASTSUM=$LS timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-include-regex "k_wta|k_hupdate" --output-format csv \
    -d $O/pmc_ls$LS/$pass -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_ls${LS}_$pass.log 2>&1 || { echo "pmc $LS $pass failed"; exit 1; }
done
python3 tools/pmc_traffic.py $O/pmc_ls$LS > $O/pmc_ls$LS.json && python3 -c "
import json; d=json.load(open('$O/pmc_ls$LS.json'))
print('LASTSUM=$LS', {k: round(v['hbm_bytes_per_launch']/1e6,1) for k,v in d.items() if isinstance(v,dict) and 'hbm_bytes_per_launch' in v})"
done
