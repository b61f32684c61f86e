"""One-rank RCCL probe: all_reduce with a pre-multiplied sum (ncclRedOpCreatePreMulSum via torch) equals x * w bitwise."""
import os, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29517")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
x = torch.randn(2_000_000, device="cuda:0")
ref = x * 0.37
y = x.clone()
dist.all_reduce(y, op=dist._make_nccl_premul_sum(0.37))
torch.cuda.synchronize()
print("premul bitwise", torch.equal(y, ref), float((y - ref).abs().max()))
dist.destroy_process_group()
