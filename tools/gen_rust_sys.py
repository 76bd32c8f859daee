#!/usr/bin/env python3
"""Generate rust/sdrgpu-sys/src/lib.rs -- the raw `extern "C"` bindings of every function,
enum constant, struct and opaque handle in include/sdrgpu.h -- the way a maintainer of the
Rust crate would write its `-sys` crate (the pattern of libsamplerate-sys, which the
reference's src/resample.rs binds).  tests/test_rust_binding.py re-parses both files and
checks that the committed output is current: every function with its argument count.

    python tools/gen_rust_sys.py            # rewrite the file
    python tools/gen_rust_sys.py --check    # exit 1 if the file is out of date
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sdrgpu.h")
OUT = os.path.join(ROOT, "rust", "sdrgpu-sys", "src", "lib.rs")

SCALARS = {"int": "c_int", "int32_t": "i32", "uint32_t": "u32", "uint8_t": "u8",
           "size_t": "usize", "float": "f32", "double": "f64", "long": "c_long",
           "char": "c_char", "void": "c_void"}


def strip_comments(src):
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def rust_type(ctype):
    """C declaration type (no name) -> Rust FFI type."""
    t = ctype.strip()
    stars = t.count("*")
    base = t.replace("*", " ").split()
    const_inner = False
    if base and base[0] == "const":
        const_inner = True
        base = base[1:]
    base = [b for b in base if b != "const"]
    name = " ".join(base)
    r = SCALARS.get(name, name)
    if stars == 0:
        return "()" if name == "void" else r
    # innermost pointer carries the const of the pointee; outer pointers are mutable
    out = ("*const " if const_inner else "*mut ") + r
    for _ in range(stars - 1):
        out = "*mut " + out
    return out


def split_params(params):
    params = params.strip()
    if params in ("", "void"):
        return []
    out = []
    for p in params.split(","):
        p = p.strip()
        m = re.match(r"(.*?)([A-Za-z_][A-Za-z0-9_]*)\s*$", p)
        ctype, name = m.group(1), m.group(2)
        if not ctype.strip():  # unnamed parameter
            ctype, name = p, "arg"
        out.append((name, ctype))
    return out


def parse(src):
    src = strip_comments(src)
    defines = re.findall(r"#define\s+(SDRGPU_[A-Z0-9_]+)\s+(\d+)", src)
    src = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    funcs = []
    for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_\s\*]*?)\b(sdrgpu_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;",
                         src):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ret = ret.split(";")[-1].split("}")[-1].strip()
        funcs.append((name, ret, split_params(params)))
    enums = []
    for m in re.finditer(r"enum\s+(\w+)\s*\{(.*?)\}", src, flags=re.S):
        for item in m.group(2).split(","):
            item = item.strip()
            if item:
                k, v = [x.strip() for x in item.split("=")]
                enums.append((m.group(1), k, v))
    structs = []
    for m in re.finditer(r"typedef\s+struct\s*\{(.*?)\}\s*(\w+)\s*;", src, flags=re.S):
        fields = []
        for decl in m.group(1).split(";"):
            decl = decl.strip()
            if not decl:
                continue
            mm = re.match(r"(.*?)([\w\s,]+)$", decl)
            # "long input_frames, output_frames" -> two fields of one type
            head = re.match(r"((?:const\s+)?[A-Za-z_]\w*\s*\**)\s*(.*)$", decl)
            ctype, names = head.group(1), head.group(2)
            for nm in names.split(","):
                nm = nm.strip()
                extra = nm.count("*")
                fields.append((nm.replace("*", "").strip(), ctype + "*" * extra))
        structs.append((m.group(2), fields))
    opaque = re.findall(r"typedef\s+struct\s+(\w+)\s+\w+\s*;", src)
    return funcs, enums, defines, structs, opaque


RUST_KEYWORDS = {"in", "type", "ref", "mod", "fn", "impl", "loop", "move", "self", "use"}


def c_layouts(structs):
    """{struct: (sizeof, [(field, offsetof), ...])} as gcc lays the header's structs out on
    this ABI (x86-64 Linux, the reference's target): a probe including sdrgpu.h is compiled
    and run.  The generated crate asserts the same numbers at compile time."""
    import tempfile
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "sdrgpu.h"', "int main(void) {"]
    for sname, fields in structs:
        lines.append(f'    printf("S {sname} %zu\\n", sizeof({sname}));')
        for fname, _ in fields:
            lines.append(f'    printf("F {sname} {fname} %zu\\n", offsetof({sname}, {fname}));')
    lines += ["    return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "probe.c"), os.path.join(d, "probe")
        open(src, "w").write("\n".join(lines) + "\n")
        import subprocess
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    lay = {}
    for line in out.splitlines():
        t = line.split()
        if t[0] == "S":
            lay[t[1]] = (int(t[2]), [])
        else:
            lay[t[1]][1].append((t[2], int(t[3])))
    return lay


def generate():
    funcs, enums, defines, structs, opaque = parse(open(HEADER).read())
    L = ["// GENERATED by tools/gen_rust_sys.py from include/sdrgpu.h -- do not edit by hand.",
         "//! Raw bindings of libsdrgpu.so (include/sdrgpu.h): the MI355X sample-stream core that",
         "//! replaces the CPU hot path of the `sdr` crate (src/filter, src/fft.rs, src/resample.rs).",
         "//! Same shape as libsamplerate-sys, the crate's only existing FFI dependency",
         "//! (Cargo.toml:24-26, bound by src/resample.rs).  Safe wrappers: ../../sdrgpu.",
         "#![allow(non_camel_case_types, non_upper_case_globals, dead_code)]",
         "",
         "use std::os::raw::{c_char, c_int, c_long, c_void};",
         ""]
    for k, v in defines:
        L.append(f"pub const {k}: c_int = {v};")
    L.append("")
    last = None
    for ename, k, v in enums:
        if ename != last:
            L.append(f"// enum {ename}")
            last = ename
        L.append(f"pub const {k}: c_int = {v};")
    L.append("")
    for o in opaque:
        L.append(f"/// opaque handle (`{o}*` in C)")
        L.append(f"#[repr(C)]\npub struct {o} {{\n    _private: [u8; 0],\n}}")
    L.append("")
    for sname, fields in structs:
        L.append("#[repr(C)]\n#[derive(Clone, Copy, Debug)]")
        L.append(f"pub struct {sname} {{")
        for fname, ftype in fields:
            L.append(f"    pub {fname}: {rust_type(ftype)},")
        L.append("}")
        L.append("")
    lay = c_layouts(structs)
    L.append("// #[repr(C)] layouts = the C compiler's (sizes / offsets from tools/gen_rust_sys.py's")
    L.append("// gcc probe of include/sdrgpu.h): a field-order or type mismatch fails to compile.")
    for sname, _ in structs:
        size, offs = lay[sname]
        L.append(f"const _: () = assert!(std::mem::size_of::<{sname}>() == {size});")
        for fname, off in offs:
            L.append(f"const _: () = assert!(std::mem::offset_of!({sname}, {fname}) == {off});")
    L.append("")
    L.append('#[link(name = "sdrgpu")]')
    L.append('extern "C" {')
    for name, ret, params in funcs:
        args = []
        for pname, ptype in params:
            pn = pname + "_" if pname in RUST_KEYWORDS else pname
            args.append(f"{pn}: {rust_type(ptype)}")
        r = rust_type(ret)
        tail = "" if r == "()" else f" -> {r}"
        line = f"    pub fn {name}({', '.join(args)}){tail};"
        if len(line) > 100:
            inner = ",\n        ".join(args)
            line = f"    pub fn {name}(\n        {inner},\n    ){tail};"
        L.append(line)
    L.append("}")
    return "\n".join(L) + "\n"


def main():
    text = generate()
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        sys.exit(0 if cur == text else 1)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    open(OUT, "w").write(text)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
