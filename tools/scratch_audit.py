"""Scratch audit of the device code: for every kernel in a hipcc -S listing, the private segment the
code object declares (.amdhsa_private_segment_fixed_size) and the scratch instructions its body
actually executes (scratch_load / scratch_store / buffer_* on the private segment).  A declared
frame with no scratch instruction is a dead frame (no memory traffic); real spills show up as
instructions.

  hipcc ... -S --cuda-device-only mapf_rollout_wide.hip -o rw.s && python tools/scratch_audit.py rw.s
"""
import re
import sys


def audit(path):
    s = open(path).read()
    rows = []
    for m in re.finditer(r"^(_Z\S+):[^\n]*$", s, re.M):
        name = m.group(1)
        end = s.find(".Lfunc_end", m.end())
        if end < 0 or not name.startswith("_Z"):
            continue
        desc = s.find(".amdhsa_kernel " + name)
        if desc < 0:
            continue
        body = s[m.end():end]
        fixed = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", s[desc:desc + 4000])
        insts = len(re.findall(r"^\s*(scratch_(load|store)\w*|buffer_(load|store)\w*[^\n]*off(en)?\b)", body, re.M))
        rows.append((name, int(fixed.group(1)) if fixed else 0, insts))
    return rows


if __name__ == "__main__":
    for path in sys.argv[1:]:
        for name, fixed, insts in audit(path):
            if fixed or insts:
                kind = "dead frame (no scratch instruction)" if insts == 0 else f"{insts} scratch instructions"
                print(f"{fixed:4d} B/lane declared  {kind:40s} {name}")
