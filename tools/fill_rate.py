"""Operand-fill rate of dc_conv_gemm per conv shape, from a per-shape breakdown (tools/conv_breakdown.py output).

Every k-chunk of every tile moves (BM + BN) x BK bf16 operands into LDS (LDS-DMA), whatever the split-K /
stream-K decomposition, so a launch fills tiles x chunks x (BM + BN) x BK x 2 bytes.  Divided by the launch time
and the 256 CUs this is the L2 -> LDS rate per CU, to be set against the measured LDS-gather rates of
MI355X_MICROARCH.md ('Indexed rows: gather into LDS': 66-73 GB/s per CU served from L2 at 72 KiB in flight).

Usage: python tools/fill_rate.py profiles/r02za/conv_breakdown_c2.txt [--top 25]
"""
import argparse
import re

# (BM, BN, BK, S) of dc_conv_gemm's algorithm table (csrc/conv_gemm.hip kAlgos), index = algo
ALGOS = [(0, 0, 0, 0), (128, 128, 64, 4), (128, 64, 64, 5), (64, 64, 64, 4), (64, 128, 64, 4), (128, 128, 64, 3),
         (128, 128, 32, 3), (128, 64, 32, 4), (64, 64, 32, 4), (256, 64, 32, 3), (128, 128, 64, 2), (128, 128, 32, 2),
         (128, 64, 64, 2), (64, 64, 64, 2), (256, 128, 32, 2), (128, 256, 32, 2), (256, 64, 64, 2), (128, 32, 64, 2),
         (64, 32, 64, 2), (64, 64, 64, 8), (128, 64, 64, 6), (64, 128, 64, 6), (64, 64, 32, 8), (64, 64, 64, 5),
         (64, 64, 64, 3)]
LINE = re.compile(r"M=\s*(\d+) N=\s*(\d+) K=\s*(\d+) mode=(\d) k=(\d) x\s*(\d+):\s*([\d.]+) us.*?([\d.]+) TF/s, "
                  r"algo \((\d+), (-?\d+)\)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("breakdown")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    rows, tot_us, tot_b = [], 0.0, 0.0
    for line in open(args.breakdown):
        m = LINE.match(line)
        if not m:
            continue
        M, N, K, _mode, _k, cnt, us, tf, a, _s = m.groups()
        M, N, K, cnt, a, us = int(M), int(N), int(K), int(cnt), int(a), float(us)
        if a == 0:
            continue  # library heuristic: tile unknown here
        bm, bn, bk, s = ALGOS[a]
        tiles = -(-M // bm) * -(-N // bn)
        fill = tiles * (K // bk) * (bm + bn) * bk * 2  # bytes per launch
        tot_us += us
        tot_b += fill * cnt
        rows.append((us, f"M={M:6d} N={N:5d} K={K:5d} x{cnt:2d} {us:7.1f} us {float(tf):6.1f} TF/s "
                         f"{bm}x{bn}x{bk} S{s}: fill {fill / 1e6:6.1f} MB/launch, "
                         f"{fill * cnt / (us * 1e-6) / 256 / 1e9:5.1f} GB/s per CU"))
    for _, r in sorted(rows, reverse=True)[:args.top]:
        print(r)
    print(f"all tuned launches: {tot_b / 1e9:.1f} GB filled in {tot_us:.0f} us = "
          f"{tot_b / (tot_us * 1e-6) / 256 / 1e9:.1f} GB/s per CU")


if __name__ == "__main__":
    main()
