"""ISA statistics of the kernels in a hipcc -S device assembly file (development tool).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude --cuda-device-only -S x.hip -o /tmp/x.s
    python tools/isa_stats.py /tmp/x.s [name-substring]
"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]

        def meta(key):
            r = re.search(re.escape(name) + r"\." + key + r", (\d+)", s)
            return r.group(1) if r else "?"
        scratch = re.search(r"\.amdhsa_kernel " + re.escape(name) + r".*?\.amdhsa_private_segment_fixed_size (\d+)",
                            s, re.S)
        print(f"{name[:70]:70s} vgpr {meta('num_vgpr')} agpr {meta('num_agpr')} scratch "
              f"{scratch.group(1) if scratch else '?'} mfma {body.count('v_mfma')} ds_read {body.count('ds_read')} "
              f"vmcnt(0) {body.count('vmcnt(0)')} s_barrier {body.count('s_barrier')} "
              f"scratch_ops {body.count('scratch_')}")


if __name__ == "__main__":
    main()
