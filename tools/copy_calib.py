"""Write-counter calibration (run under ``rocprofv3 --kernel-trace --pmc
TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum``): a device copy
of exactly 1.6 GB (reads 1.6 GB, writes 1.6 GB), three dispatches.  The
known bytes over the copy kernel's request counts give the bytes per read /
write request on this part; tools/pmc_summary.py prints the counts."""
import torch


def main():
    dev = torch.device("cuda", 0)
    n = 400_000_000
    x = torch.ones(n, dtype=torch.float32, device=dev)
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()
    print(f"copy bytes per dispatch: read {n * 4} write {n * 4}")


if __name__ == "__main__":
    main()
