import time, numpy as np, torch, sys
sys.path.insert(0, '.')
import litenetlibpp_amd as P
torch.cuda.init()
rng = np.random.default_rng(1)
for n in (64, 1024, 4096, 65536):
    lens = rng.integers(100, 1400, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    buf = torch.empty(int(off[-1]), dtype=torch.uint8).pin_memory().numpy()
    buf[:] = rng.integers(0, 256, buf.size, dtype=np.uint8)
    for f in (P.inbound_filter_host, P.batch_host):
        f(buf, off, 0)
        t = time.perf_counter(); R = 50
        for _ in range(R): f(buf, off, 0)
        dt = (time.perf_counter() - t) / R
        print(f.__name__, n, f"{dt*1e6:.1f} us/call", f"{off[-1]/dt/1e9:.2f} GB/s", flush=True)
