"""Instruction-level diff of one kernel between two `hipcc --offload-device-only -S` outputs.
   python tools/isa_diff.py OLD.s NEW.s KERNEL_SYMBOL  (labels and comments ignored)"""
import difflib
import re
import sys


def body(path, name):
    s = open(path).read()
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    out = []
    for l in s[i:j].splitlines()[1:]:
        t = l.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        out.append(re.sub(r"\.LBB\d+_\d+", "L", t))
    return out


a, b = body(sys.argv[1], sys.argv[3]), body(sys.argv[2], sys.argv[3])
d = [l for l in difflib.unified_diff(a, b, lineterm="", n=0) if not l.startswith("@@")]
print(f"{len(a)} -> {len(b)} instructions, {len(d)} diff lines")
print("\n".join(d[:int(sys.argv[4]) if len(sys.argv) > 4 else 60]))
