"""Scan hipcc's gfx950 assembly for a 16/12-byte vector store whose data
VGPRs the very next VALU instruction overwrites (no wait state between).
hipcc 7.2 emitted that after __builtin_amdgcn_raw_buffer_store_b128 (the
store then reads some lanes' new values: archive:cgu_debug.py); BufSeg stores
therefore use global stores. Usage: python tools/store_hazard_scan.py [src.hip ...]
(default: every krylov_amd/csrc/*.hip); prints hits per kernel, exit 1 if any."""
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def scan(asm):
    hits, kern = {}, None
    lines = asm.split("\n")
    for i, l in enumerate(lines):
        if l.startswith("_Z") and ": ;" in l:
            kern = l.split(":")[0]
        s = l.strip()
        if re.match(r"(buffer|global|flat)_store_dwordx(3|4)", s) and i + 1 < len(lines):
            parts = s.split()
            data = parts[1].rstrip(",") if s.startswith("buffer") else parts[2].rstrip(",")
            nxt = lines[i + 1].strip()
            if nxt.startswith("v_") and len(nxt.split()) > 1 and regs(nxt.split()[1].rstrip(",")) & regs(data):
                hits[kern] = hits.get(kern, 0) + 1
    return hits


def main(srcs):
    bad = 0
    for src in map(os.path.abspath, srcs):
        with tempfile.NamedTemporaryFile(suffix=".s") as f:
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                                   "-ffp-contract=off", "--cuda-device-only", "-S", src, "-o", f.name],
                                  cwd=os.path.dirname(src), stderr=subprocess.DEVNULL)
            hits = scan(open(f.name).read())
        print(os.path.basename(src), sum(hits.values()), list(hits.items())[:5])
        bad += sum(hits.values())
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or sorted(glob.glob(os.path.join(REPO, "krylov_amd", "csrc", "*.hip")))))
