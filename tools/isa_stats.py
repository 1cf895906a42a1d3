"""Instruction counts of the kernels in a HIP object or shared library whose
name contains every comma-separated substring: python tools/isa_stats.py
file.{o,so} gemm_bf16x6w[,W6Cfg] [--dump out.s]"""
import os
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def code_objects(path):
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs, at = [], data.find(magic)
    while at >= 0:
        n = struct.unpack_from("<Q", data, at + 24)[0]
        p = at + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                objs.append(data[at + off:at + off + size])
        at = data.find(magic, p)
    return objs


def main():
    path, want = sys.argv[1], sys.argv[2].split(",")
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    text = ""
    for co in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(co)
        text += subprocess.run([OBJDUMP, "-d", "--demangle", f.name], capture_output=True, text=True).stdout
        os.unlink(f.name)
    out = []
    for fn in re.split(r"\n(?=[0-9a-f]{16} <)", text):
        m = re.match(r"[0-9a-f]{16} <(.*)>:", fn)
        if not m or not all(w in m.group(1) for w in want):
            continue
        lines = [l for l in fn.split("\n")[1:] if l.strip()]
        c = lambda pat: sum(1 for l in lines if re.search(pat, l))
        valu = c(r"\bv_(?!mfma|accvgpr)")
        print(m.group(1)[:120])
        print(f"   instr {len(lines)} mfma {c(r'v_mfma')} accvgpr_read {c(r'v_accvgpr_read')} "
              f"accvgpr_write {c(r'v_accvgpr_write')} accvgpr_mov {c(r'v_accvgpr_mov')} scratch {c(r'scratch_')} "
              f"ds_read {c(r'ds_read')} ds_write {c(r'ds_write')} global_load {c(r'global_load')} "
              f"global_store {c(r'global_store')} s_nop {c(r's_nop')} s_waitcnt {c(r's_waitcnt')} "
              f"s_barrier {c(r's_barrier')} valu {valu}")
        out.append(fn)
    if dump:
        open(dump, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
