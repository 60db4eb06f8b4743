"""Summarise a rocprofv3 --stats kernel_stats.csv (per-step when --steps given)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print("%-70s %6s %9s %9s %6s" % ("kernel", "calls", "avg_us", "ms/step", "%"))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    name = r['Name'].replace('void ', '')[:70]
    print("%-70s %6s %9.1f %9.3f %6.2f" % (name, r['Calls'], float(r['AverageNs']) / 1e3,
                                          float(r['TotalDurationNs']) / 1e6 / steps,
                                          100 * float(r['TotalDurationNs']) / tot))
print("total kernel time per step: %.3f ms" % (tot / 1e6 / steps))
# every GEMM tile kernel of the product (bf16 and fp8; bench.py GEMM_FAMILY
# is the bf16 subset the live roofline times)
FAMILY = ("gemm_bf16_kernel", "gemm256_bf16_kernel", "gemm256s_bf16_kernel", "gemm256_wgrad_kernel",
          "gemm256s_wgrad_kernel", "gemm64_bf16_kernel", "gemm_skinny_bf16_kernel",
          "gemm256_fp8_kernel", "gemm256s_fp8_kernel")
fam = [r for r in rows if r['Name'].replace('void ', '').startswith(FAMILY)]
red = [r for r in rows if r['Name'].startswith("splitk_reduce_kernel")]
if fam:
    calls = sum(int(r['Calls']) for r in fam)
    ns = sum(float(r['TotalDurationNs']) for r in fam + red)
    print("smer_gemm family (tile kernels + split-K reduce): %d calls, %.2f us per smer_gemm call, "
          "%.3f ms/step" % (calls, ns / 1e3 / calls, ns / 1e6 / steps))
