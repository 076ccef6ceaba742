import time, torch, sys
sys.path.insert(0, '/root/repo')
import svdsolver_amd as S
n, b = 8192, 32
dev = torch.device('cuda', 0)
mats = [torch.rand((n, n), dtype=torch.float64, device=dev) * 5 for _ in range(4)]
S.ge2band(mats[0], b); torch.cuda.synchronize()
for i in range(1, 4):
    t0 = time.perf_counter(); S.ge2band(mats[i], b, sync=False); t1 = time.perf_counter()
    torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"enqueue {1e3*(t1-t0):.1f} ms, total {1e3*(t2-t0):.1f} ms", flush=True)
