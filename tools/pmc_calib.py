"""Known-byte kernels for calibrating FETCH_SIZE / WRITE_SIZE on this box.

Run under each PMC pass beside the bench (tools/pmc_traffic.py reads both):
  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_cal -o run --output-format csv -- python tools/pmc_calib.py
Each kernel moves exactly N bytes in and N bytes out (N = 1 GiB, > Infinity Cache).
"""
import torch

N = 1 << 30


def main():
    src = torch.empty(N, dtype=torch.uint8, device="cuda")
    src.fill_(7)
    dst = torch.empty_like(src)
    for _ in range(3):
        torch.bitwise_not(src, out=dst)  # elementwise: N read + N written, 16-B vector accesses
    torch.cuda.synchronize()
    print("calib bytes", N)


if __name__ == "__main__":
    main()
