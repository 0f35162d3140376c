"""Per-kernel instruction statistics of a hipcc -save-temps gfx950 assembly file (diagnosis only).

    python tools/isa_stats.py /tmp/kernels-hip-amdgcn-amd-amdhsa-gfx950.s k_spmv_vibm"""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
s = open(path).read()
for m in re.finditer(r"^(_Z\S*" + pat + r"\S*):\s", s, re.M):
    name = m.group(1)
    st = m.end()
    en = s.index(".Lfunc_end", st)
    body = s[st:en]
    meta = s[en:en + 4000]

    def g(k):
        mm = re.search(r"; " + k + r":\s+(\d+)", meta)
        return mm.group(1) if mm else "?"

    cnt = lambda p: len(re.findall(p, body))
    lg0 = cnt(r"lgkmcnt\(0\)")
    print(f"{name[:90]}\n   lines {body.count(chr(10))} v_mul_f64 {cnt(r'v_mul_f64')} v_add_f64 {cnt(r'v_add_f64')} "
          f"s_load {cnt(r's_load_dword')} s_buffer {cnt(r's_buffer_load')} ds_read {cnt(r'ds_read')} "
          f"lgkm0 {lg0} waitcnt {cnt(r's_waitcnt')} scratch {cnt(r'scratch_')} "
          f"readlane {cnt(r'v_readlane|v_writelane')} vgpr {g('NumVgprs')} sgpr {g('NumSgprs')} "
          f"scratch_bytes {g('ScratchSize')} occupancy {g('Occupancy')}")
