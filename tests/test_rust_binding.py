"""The Rust side of the drop-in boundary, checked on CPU (no Rust toolchain in this image):
rust/sdrgpu-sys/src/lib.rs declares every function of include/sdrgpu.h with its argument
count, the generated file is current, and every `sys::sdrgpu_*` call in the crate-side
wrapper rust/sdr-gpu/gpu.rs names a declared function with the right number of arguments.
The D = 1 FIR drop-in keeps `Fir`'s `Output = A` (src/filter/fir.rs:21-23)."""
import os
import re
import subprocess
import sys

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sdrgpu.h")
SYS = os.path.join(ROOT, "rust", "sdrgpu-sys", "src", "lib.rs")
GPU = os.path.join(ROOT, "rust", "sdr-gpu", "gpu.rs")


def split_top(s):
    """Split on commas outside (), [], <> and {}."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{<":
            depth += 1
        elif ch in ")]}>":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [x for x in (o.strip() for o in out) if x]


def header_functions():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    src = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    funcs = {}
    for m in re.finditer(r"\b(sdrgpu_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src):
        p = m.group(2).strip()
        funcs[m.group(1)] = 0 if p in ("", "void") else len(split_top(p))
    return funcs


def rust_sys_functions():
    src = open(SYS).read()
    funcs = {}
    for m in re.finditer(r"pub fn (sdrgpu_[a-z0-9_]+)\s*\((.*?)\)\s*(->[^;]*)?;", src, flags=re.S):
        funcs[m.group(1)] = len(split_top(m.group(2).replace("->", "")))
    return funcs


def test_generated_sys_file_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_rust_sys.py"), "--check"])
    assert r.returncode == 0, "rust/sdrgpu-sys/src/lib.rs is stale: run tools/gen_rust_sys.py"


def test_sys_crate_declares_every_header_function():
    h, r = header_functions(), rust_sys_functions()
    assert len(h) > 100
    assert set(h) == set(r), (set(h) ^ set(r))
    bad = {n: (h[n], r[n]) for n in h if h[n] != r[n]}
    assert not bad, bad
    src = open(SYS).read()
    assert '#[link(name = "sdrgpu")]' in src and 'extern "C"' in src
    for s in ("sdrgpu_pll_params", "sdrgpu_biquad_design", "sdrgpu_src_data"):
        assert re.search(r"#\[repr\(C\)\]\s*#\[derive\(Clone, Copy, Debug\)\]\s*pub struct " + s, src)


def test_wrapper_calls_match_the_header():
    h = header_functions()
    src = open(GPU).read()
    calls = []
    for m in re.finditer(r"sys::(sdrgpu_[a-z0-9_]+)\s*\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        calls.append((m.group(1), len(split_top(src[m.end():i - 1]))))
    assert len(calls) > 30
    bad = [(n, k, h.get(n)) for n, k in calls if h.get(n) != k]
    assert not bad, bad


def test_d1_fir_drop_in_keeps_output_a():
    src = open(GPU).read()
    m = re.search(r"impl<A: GpuSample> Filter<A> for GpuFir<A> \{\s*type Output = (\w+);", src)
    assert m and m.group(1) == "A"
    m = re.search(r"impl<A: GpuSample, C: GpuSample> FilterDesign<A> for GpuFirD<C> \{\s*"
                  r"type Output = (\w+);\s*type Filter = GpuFir<A>;", src)
    assert m and m.group(1) == "A"
    # the decimating form is the one whose per-sample output is Option<A>
    assert re.search(r"Filter<A> for GpuFirDecim<A> \{\s*type Output = Option<A>;", src)


RUST_SIZE_ALIGN = {"c_int": 4, "i32": 4, "u32": 4, "u8": 1, "usize": 8, "f32": 4, "f64": 8,
                   "c_long": 8, "c_char": 1}


def rust_structs():
    src = open(SYS).read()
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*#\[derive[^\]]*\]\s*pub struct (\w+) \{(.*?)\}", src,
                         flags=re.S):
        out[m.group(1)] = re.findall(r"pub (\w+): ([^,]+),", m.group(2))
    return out


def repr_c_layout(name, structs):
    """(size, align, {field: offset}) of a #[repr(C)] struct from its Rust field types, by the
    C layout rules repr(C) follows (x86-64: pointers and c_long are 8 bytes)."""
    off, align, offs = 0, 1, {}
    for fname, ftype in structs[name]:
        ftype = ftype.strip()
        if ftype.startswith("*"):
            sz = al = 8
        elif ftype in RUST_SIZE_ALIGN:
            sz = al = RUST_SIZE_ALIGN[ftype]
        else:
            sz, al, _ = repr_c_layout(ftype, structs)
        off = (off + al - 1) // al * al
        offs[fname] = off
        off += sz
        align = max(align, al)
    return (off + align - 1) // align * align, align, offs


def test_sys_struct_layouts_match_the_c_header():
    """Advisor finding r3: the #[repr(C)] structs' field order and Rust types must lay out as
    the C compiler lays out include/sdrgpu.h's structs.  lib.rs carries the gcc-measured
    sizes / offsets as compile-time asserts (generated, and checked current above); here the
    layout implied by the Rust field types is computed independently and compared with them,
    and the field order with the header's."""
    src = open(SYS).read()
    structs = rust_structs()
    assert set(structs) >= {"sdrgpu_pll_params", "sdrgpu_biquad_design", "sdrgpu_src_data",
                            "sdrgpu_comm_op"}
    sizes = dict(re.findall(r"size_of::<(\w+)>\(\) == (\d+)\)", src))
    offsets = re.findall(r"offset_of!\((\w+), (\w+)\) == (\d+)\)", src)
    assert set(sizes) == set(structs)
    for name in structs:
        size, _, offs = repr_c_layout(name, structs)
        assert size == int(sizes[name]), (name, size, sizes[name])
        c_offs = [(f, int(o)) for s, f, o in offsets if s == name]
        assert [f for f, _ in c_offs] == [f for f, _ in structs[name]], name   # same order
        assert all(offs[f] == o for f, o in c_offs), (name, offs, c_offs)
