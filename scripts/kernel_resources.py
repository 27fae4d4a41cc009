"""Per-kernel VGPR/AGPR/scratch/occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.
Usage: python scripts/kernel_resources.py <file.hip> [extra hipcc flags...]"""
import re
import subprocess
import sys


def main() -> None:
    src, extra = sys.argv[1], sys.argv[2:]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", *extra, "-c", src, "-o", "/tmp/_kr.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?)(?: \[-Rpass)", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            cur = {"name": re.sub(r"^_Z\w*?(gemm_fused_kernel|[a-z_]+_kernel)", r"\1", txt.split(":", 1)[1].strip())[:60]}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        print(f"{r['name']:60s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>4} "
              f"scratch={r.get('ScratchSize [bytes/lane]','?'):>3} occ={r.get('Occupancy [waves/SIMD]','?')}")


if __name__ == "__main__":
    main()
