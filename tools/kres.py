"""Per-kernel resources from a device .s (hipcc --cuda-device-only -S):
python tools/kres.py file.s [substring]"""
import re, sys
s = open(sys.argv[1]).read()
meta = s[s.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    name = f.get("name", "?")
    if len(sys.argv) > 2 and sys.argv[2] not in name:
        continue
    print("%-60s vgpr %4s agpr %4s sgpr %4s lds %6s spill %s" % (
        name[:60], f.get("vgpr_count"), f.get("agpr_count"), f.get("sgpr_count"),
        f.get("group_segment_fixed_size"), f.get("vgpr_spill_count")))
