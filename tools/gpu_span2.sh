bash tools/gpu_span.sh && timeout -k 10 300 python3 tools/kvariants.py run --names base,span_nofold,bucketed --rounds 6 --workloads csr:1048576:64:1400
