"""Per-kernel register / spill / LDS usage of one HIP source for gfx950 (compiler remarks):
    python scripts/kres.py gru_mpi_cuda_amd/csrc/kernels/gru_seq.hip [name-filter]"""
import re, subprocess, sys
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Igru_mpi_cuda_amd/csrc",
       "-I/opt/rocm/include", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "LDS Size \\[bytes/block\\]"):
        m = re.search(r"\s" + key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split(" [")[0].replace("\\", "")] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f'{r["name"][:70]:70s} vgpr={r.get("VGPRs")} agpr={r.get("AGPRs")} vspill={r.get("VGPRs Spill")} '
              f'sspill={r.get("SGPRs Spill")} lds={r.get("LDS Size")}')
