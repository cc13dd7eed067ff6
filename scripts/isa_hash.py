#!/usr/bin/env python3
"""Per-kernel hashes of gfx950 device assembly (hipcc --cuda-device-only -S), for "this change leaves
kernel X's machine code untouched" checks: label numbers are normalized (they shift when kernels are
added), comments and directives dropped.

    python3 scripts/isa_hash.py build.s            -> "<hash> <kernel>" per kernel
    python3 scripts/isa_hash.py a.s b.s            -> kernels present in both whose code differs
    python3 scripts/isa_hash.py a.s b.s --defaulted-last   (b's kernels have one more defaulted template
                                                            argument and a trailing NeeParams argument)
"""
import hashlib
import re
import sys


def norm(s):
    # .LBB<function>_<block>: the function number shifts when kernels are added, the block does not
    return re.sub(r"\.Ltmp\d+", ".Ltmp", re.sub(r"\.LBB\d+_(\d+)", r".LBB_\1", s))


def kernels(path):
    out, name, body, meta = {}, None, [], {}
    for line in open(path):
        m = re.match(r"^(_Z[^\s:]+):", line)
        if m and "@function" not in line:
            name, body = m.group(1), []
            continue
        if name is None:
            continue
        if line.startswith(".Lfunc_end"):
            out[name] = body
            name = None
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith("."):
            if s.startswith(".LBB") or s.startswith(".Ltmp"):
                body.append(norm(s))
            continue
        body.append(norm(s))
    return {k: hashlib.sha1("\n".join(v).encode()).hexdigest()[:12] for k, v in out.items()}


def main():
    a = kernels(sys.argv[1])
    if len(sys.argv) == 2:
        for k, h in sorted(a.items()):
            print(h, k[:140])
        return
    b = kernels(sys.argv[2])
    if len(sys.argv) > 3 and sys.argv[3] == "--defaulted-last":
        # b's kernels gained a defaulted last template argument (false) and a trailing NeeParams
        # argument: map their names back to a's
        def back(k):
            if not k.endswith("NS_9NeeParamsE"):
                return k
            k = k[: -len("NS_9NeeParamsE")]
            i = k.rfind("Lb0EEEv")
            return k[:i] + k[i + 4:] if i >= 0 else k
        b = {back(k): v for k, v in b.items()}
    same = diff = 0
    for k in sorted(set(a) & set(b)):
        if a[k] == b[k]:
            same += 1
        else:
            diff += 1
            print("DIFFERS", k[:160])
    print(f"{same} identical, {diff} differ, {len(set(b) - set(a))} new, {len(set(a) - set(b))} gone")


if __name__ == "__main__":
    main()
