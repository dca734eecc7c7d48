# round 5: tiled flat XOR (one workgroup per tile of the batch) against the
# persistent grid, config-2-shaped XOR batch (kvariants base = experiments build)
set -o pipefail
out=gpurun_out/r05l_xor_flat_tiles.log
: > $out
for v in 6:8 6:1000000 11:8 12:8 13:8 14:8 15:8 6:8; do
  LNL_XOR_FLAT=${v%%:*} LNL_XOR_FLAT_WG=${v##*:} timeout -k 10 100 python tools/kvariants.py run --names base --rounds 12 \
    --workloads xor:1048576:1400,xor:4194304:256 --out gpurun_out/r05l_tmp.json > /tmp/r05l.log 2>&1 || { cat /tmp/r05l.log; exit 1; }
  grep base@ /tmp/r05l.log | sed "s/^/flat=$v /" >> $out
done
cat $out
