import sys, json, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import test_gpu_kernels as T
gpu = torch.device("cuda:0")
for seed, n in [(0, 3000), (3, 5000)]:
    cpu_raw, cpu_ok, gpu_raw, gpu_ok = T._parse_both(gpu, n=n, seed=seed)
    a, b = cpu_raw.to_pylist(), gpu_raw.to_pylist()
    bad = [i for i in range(len(a)) if a[i] != b[i]]
    print("seed", seed, "mismatch rows", len(bad), "ok equal", torch.equal(cpu_ok.cpu(), gpu_ok.cpu()))
    for i in bad[:3]:
        print(T._records(n, seed)[i][:300])
        print(" cpu", a[i]); print(" gpu", b[i])
