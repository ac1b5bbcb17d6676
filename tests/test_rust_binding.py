"""The Rust binding in INTEGRATION.md (the `extern "C"` block a RustDDS maintainer would
commit, bindgen-equivalent) against include/rtps_rx.h, on the CPU.

There is no Rust toolchain in this image, so the block cannot be compiled here.  These
tests hold it to the header instead:
  * every function the header declares is in the block, with the same arity and the same
    parameter widths (pointer / 1 / 2 / 4 / 8 bytes) and return width, and the block
    declares nothing the header does not;
  * every struct the header defines is a #[repr(C)] struct of the block, and its size and
    every field offset (computed with the C layout rules from the Rust field types) equal
    what gcc reports for the header (a sizeof / offsetof probe compiled here);
  * every opaque handle of the header is an uninhabited enum of the block.
Reference boundary: rtps/message.rs:64 (Message::read_from_buffer) and
io_uring/rtps/message_receiver.rs:232 (handle_received_packet_2), the calls the block's
rtps_rx_parse_batch replaces."""
import os
import re
import subprocess


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rtps_rx.h")

C_WIDTH = {"uint8_t": 1, "int8_t": 1, "char": 1, "uint16_t": 2, "int16_t": 2, "uint32_t": 4, "int32_t": 4,
           "int": 4, "uint64_t": 8, "int64_t": 8, "void": 0}
R_PRIM = {"u8": (1, 1), "i8": (1, 1), "u16": (2, 2), "i16": (2, 2), "u32": (4, 4), "i32": (4, 4),
          "c_int": (4, 4), "u64": (8, 8), "i64": (8, 8), "f32": (4, 4), "f64": (8, 8)}


def _strip_c(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return "\n".join(line for line in text.splitlines() if not line.lstrip().startswith("#"))


def header_functions():
    src = _strip_c(open(HEADER).read())
    out = {}
    for m in re.finditer(r"(?:^|[;}])\s*((?:const\s+)?\w+\s*\**)\s*\b(rtps_\w+)\s*\(([^()]*)\)\s*;", src, re.M):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        widths = []
        if params and params != "void":
            for prm in params.split(","):
                prm = prm.strip()
                if "*" in prm or "[" in prm:
                    widths.append(8)
                else:
                    base = prm.replace("const", "").split()[0]
                    widths.append(C_WIDTH[base])
        rw = 8 if "*" in ret else C_WIDTH[ret.replace("const", "").strip()]
        out[name] = (widths, rw)
    return out


def header_structs():
    src = _strip_c(open(HEADER).read())
    defined = set(re.findall(r"typedef\s+struct\s+(\w+)\s*\{", src))
    opaque = {a for a, b in re.findall(r"typedef\s+struct\s+(\w+)\s+(\w+)\s*;", src) if a == b}
    return defined, opaque


def rust_block():
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"```rust\n(.*?)```", text, re.S)
    assert m, "INTEGRATION.md has no ```rust block"
    code = re.sub(r"/\*.*?\*/", " ", m.group(1), flags=re.S)
    return re.sub(r"//[^\n]*", " ", code)


def _split_top(s):
    """Split on commas outside brackets / parentheses / angle brackets."""
    parts, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([<":
            depth += 1
        elif ch in ")]>":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return [p.strip() for p in parts if p.strip()]


def rust_functions(code):
    out = {}
    for m in re.finditer(r"pub fn (\w+)\(([^()]*)\)\s*(?:->\s*([^;]+))?;", code):
        name, params, ret = m.group(1), m.group(2), (m.group(3) or "").strip()
        widths = []
        for prm in _split_top(params):
            ty = prm.split(":", 1)[1].strip()
            widths.append(8 if ty.startswith("*") else R_PRIM[ty][0])
        rw = 0 if not ret else 8 if ret.startswith("*") else R_PRIM[ret][0]
        out[name] = (widths, rw)
    return out


def rust_structs(code):
    structs = {}
    for m in re.finditer(r"#\[repr\(C\)\](?:\s*#\[derive\([^)]*\)\])?\s*pub struct (\w+)\s*\{(.*?)\}", code, re.S):
        fields = []
        for f in _split_top(m.group(2)):
            name, ty = f.split(":", 1)
            fields.append((name.replace("pub", "").strip(), ty.strip()))
        structs[m.group(1)] = fields
    types = dict(re.findall(r"pub type (\w+)\s*=\s*([^;]+);", code))
    enums = set(re.findall(r"pub enum (\w+)\s*\{\s*\}", code))
    return structs, types, enums


def rust_layout(structs, types):
    memo = {}

    def size_align(ty):
        ty = ty.strip()
        if ty in types:
            return size_align(types[ty])
        if ty.startswith("*") or ty.startswith("Option<"):
            return 8, 8
        if ty in R_PRIM:
            return R_PRIM[ty]
        m = re.fullmatch(r"\[(.+);\s*(\d+)\]", ty)
        if m:
            s, a = size_align(m.group(1))
            return s * int(m.group(2)), a
        return layout(ty)[0:2]

    def layout(name):
        if name not in memo:
            off, align, offs = 0, 1, {}
            for fname, fty in structs[name]:
                s, a = size_align(fty)
                off = (off + a - 1) // a * a
                offs[fname] = off
                off += s
                align = max(align, a)
            memo[name] = ((off + align - 1) // align * align, align, offs)
        return memo[name]

    return {n: (layout(n)[0], layout(n)[2]) for n in structs}


def c_name(rust):
    return "rtps" + re.sub(r"([A-Z])", lambda m: "_" + m.group(1).lower(), rust[4:])


def test_every_header_function_is_bound_with_its_arity_and_widths():
    hf = header_functions()
    rf = rust_functions(rust_block())
    assert len(hf) >= 45, f"header parse found only {len(hf)} functions"
    missing = sorted(set(hf) - set(rf))
    extra = sorted(set(rf) - set(hf))
    assert not missing, f"header functions missing from the Rust block: {missing}"
    assert not extra, f"Rust block declares functions the header does not: {extra}"
    bad = {n: (hf[n], rf[n]) for n in hf if hf[n] != rf[n]}
    assert not bad, f"arity / width mismatch (header, rust): {bad}"


def test_every_struct_matches_the_c_layout(tmp_path):
    code = rust_block()
    structs, types, enums = rust_structs(code)
    defined, opaque = header_structs()
    rust_c = {c_name(n): n for n in structs}
    assert not sorted(defined - set(rust_c)), f"header structs missing from the block: {sorted(defined - set(rust_c))}"
    assert not sorted(set(rust_c) - defined), f"block structs not in the header: {sorted(set(rust_c) - defined)}"
    assert {c_name(e) for e in enums} == opaque, (sorted(opaque), sorted(enums))
    lay = rust_layout(structs, types)
    probe = ['#include <stdio.h>', '#include <stddef.h>', '#include "rtps_rx.h"', "int main(void) {"]
    for rn, (size, offs) in lay.items():
        cn = c_name(rn)
        probe.append(f'  printf("{rn} #size %zu\\n", sizeof({cn}));')
        for f in offs:
            probe.append(f'  printf("{rn} {f} %zu\\n", offsetof({cn}, {f}));')
    probe += ["  return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(probe))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)],
                   check=True, capture_output=True)
    got = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        a, b, v = line.split()
        got[(a, b)] = int(v)
    bad = []
    for rn, (size, offs) in lay.items():
        if got[(rn, "#size")] != size:
            bad.append(f"{rn}: size rust {size} != C {got[(rn, '#size')]}")
        for f, o in offs.items():
            if got[(rn, f)] != o:
                bad.append(f"{rn}.{f}: offset rust {o} != C {got[(rn, f)]}")
    assert not bad, bad


def test_the_check_fails_on_a_missing_export():
    """The check is not vacuous: dropping one declaration from the block is caught."""
    code = rust_block().replace("pub fn rtps_rx_frag_reset(", "pub fn renamed_away(")
    rf = rust_functions(code)
    assert "rtps_rx_frag_reset" in set(header_functions()) - set(rf)
