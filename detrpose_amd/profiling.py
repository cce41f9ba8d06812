"""Kernel names as rocprofv3 reports them, reduced to one canonical form, so a plan's launches
(Plan.kernel_of: the dispatcher's choice from dp_conv2d_describe, else the C entry point) can be
matched with `--kernel-trace --stats` summaries and PMC counter rows.

rocprofv3 prints some instantiations demangled ("void (anonymous namespace)::conv_halo_kernel<8,
4, ...>(dp_conv_desc, ...)") and others mangled ("_ZN12_GLOBAL__N_118conv_stream_kernelILi256E...
DF16bLi0EEEv12dp_conv_desciiii"); both become "conv_stream_kernel<256, ..., bf16, 0>".
"""
from __future__ import annotations

import re

_TOK = re.compile(r"Li(-?\d+)E|Lb([01])E|(DF16b)|(f)(?=[LE])")


def _demangle_args(s: str) -> list[str]:
    out, i = [], 0
    while i < len(s):
        m = _TOK.match(s, i)
        if not m:
            break
        if m.group(1) is not None:
            out.append(m.group(1))
        elif m.group(2) is not None:
            out.append("true" if m.group(2) == "1" else "false")
        elif m.group(3):
            out.append("bf16")
        else:
            out.append("float")
        i = m.end()
    return out


def canonical_kernel_name(name: str) -> str:
    name = name.strip().strip('"')
    m = re.match(r"_ZN12_GLOBAL__N_1\d+(\w+?)I(.*)EEv", name)
    if m:
        return f"{m.group(1)}<{', '.join(_demangle_args(m.group(2)))}>"
    m = re.match(r"_ZN12_GLOBAL__N_1\d+(\w+?)E", name)
    if m:
        return m.group(1)
    name = re.sub(r"^void\s+", "", name)
    name = name.replace("(anonymous namespace)::", "")
    # cut the parameter list: the first "(" outside template brackets
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    return name.replace("bool _Accum", "bf16").replace("__bf16", "bf16").strip()


def kernel_family(canonical: str) -> str:
    """The kernel template / function name without arguments."""
    return canonical.split("<", 1)[0]
