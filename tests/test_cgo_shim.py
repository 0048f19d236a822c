"""The cgo shim (network-stack_amd/go/transport/tcp/*_nsx.go) tied to the C ABI mechanically.

No Go toolchain exists in this container or on the GPU box, so the shim cannot be compiled
by cgo here. Instead this test does what cgo's type check would do, from the sources:
  - every `C.nsx_*` call in the shim names a function declared in include/nsx_csum.h and exported by
    libnsx_csum.so, with the argument count the header declares;
  - every argument's Go type (inferred from the shim's own casts and declarations: `(*C.uint8_t)(x)`,
    `C.uint64_t(n)`, `var partial *C.uint32_t`, `&p` of an `unsafe.Pointer`, ...) is exactly the C parameter
    type cgo would require (const stripped; `void*` <-> unsafe.Pointer) — Go has no implicit conversions, so a
    header change that alters a parameter's type or position breaks this test as it would break `go build`;
  - every `C.NSX_*` constant and `C.*` type the shim names exists in the header;
  - a C translation unit making exactly those calls with exactly those argument types compiles under
    -Wall -Werror and links against the library.
A header change that breaks the shim therefore fails `pytest -m "not gpu"`."""
import os
import re
import subprocess

import pytest

import nsx
from conftest import ROOT

GO_DIR = os.path.join(ROOT, "network-stack_amd", "go", "transport", "tcp")
HEADER = os.path.join(ROOT, "include", "nsx_csum.h")
SHIM_FILES = ("checksum_nsx.go", "batch_nsx.go", "rx_nsx.go", "build_nsx.go")


def _norm(t: str) -> str:
    t = re.sub(r"\bconst\b", "", t)
    t = re.sub(r"\s+", "", t)
    return "void*" if t == "nsx_stream_t" else t


def header_prototypes() -> dict:
    """name -> (return type, [param C types]) for every function include/nsx_csum.h declares."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    protos = {}
    for m in re.finditer(r"^\s*((?:const\s+)?[a-z_0-9]+\s*\*?)\s*(nsx_[a-z_0-9]+)\s*\(([^)]*)\)\s*;", src, re.M):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        types = []
        if params and params != "void":
            for p in params.split(","):
                p = p.strip()
                pm = re.match(r"^(.*?[\s*])([A-Za-z_][A-Za-z_0-9]*)$", p)
                assert pm, (name, p)
                types.append(_norm(pm.group(1)))
        protos[name] = (_norm(ret), types)
    return protos


def header_typedefs() -> set:
    """The struct typedef names include/nsx_csum.h declares (cgo's C.<name>)."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return set(re.findall(r"typedef\s+struct\s*\{[^}]*\}\s*(\w+)\s*;", src))


def header_constants() -> set:
    return set(re.findall(r"^#define\s+(NSX_[A-Z0-9_]+)", open(HEADER).read(), re.M))


def _split_args(s: str) -> list:
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _close(src: str, i: int) -> int:
    """Index of the parenthesis closing the one at src[i]."""
    depth = 0
    for j in range(i, len(src)):
        depth += {"(": 1, ")": -1}.get(src[j], 0)
        if depth == 0:
            return j
    raise AssertionError("unbalanced parentheses")


def go_to_c(gt: str) -> str:
    """A Go type as cgo sees it -> the C type it stands for."""
    gt = gt.strip()
    if gt.startswith("*"):
        return go_to_c(gt[1:]) + "*"
    if gt == "unsafe.Pointer":
        return "void*"
    m = re.fullmatch(r"C\.(\w+)", gt)
    assert m, f"not a C type: {gt!r}"
    return m.group(1)


class GoFile:
    """Just enough of a Go source file to type the arguments of its C calls."""

    def __init__(self, path: str):
        self.path = path
        self.src = re.sub(r"//[^\n]*", "", open(path).read())
        self.vars, self.funcs, self.fields = {}, {}, {}
        for m in re.finditer(r"\bvar\s+(\w+)\s+(\*?[\w.]+)", self.src):
            self.vars[m.group(1)] = m.group(2)
        for m in re.finditer(r"^\s*func\s+(?:\([^)]*\)\s*)?(\w+)\s*\(([^)]*)\)\s*(\*?[\w.]+)?\s*\{", self.src, re.M):
            if m.group(3):
                self.funcs[m.group(1)] = m.group(3)
        for m in re.finditer(r"^\s+(\w+)\s+(\*?unsafe\.Pointer|\*?C\.\w+)\s*$", self.src, re.M):
            self.fields[m.group(1)] = m.group(2)
        # short declarations `a, b := E1, E2` (also inside `if x := ...;`)
        for m in re.finditer(r"([\w, ]+?)\s*:=\s*", self.src):
            names = [x.strip() for x in m.group(1).split(",")]
            j, depth = m.end(), 0  # the right-hand side: up to a newline, ';' or '{' outside parentheses
            while j < len(self.src) and not (depth == 0 and self.src[j] in "\n;{"):
                depth += {"(": 1, ")": -1}.get(self.src[j], 0)
                j += 1
            exprs = _split_args(self.src[m.end():j].strip())
            if len(names) == len(exprs):
                for nm, ex in zip(names, exprs):
                    if re.fullmatch(r"\w+", nm):
                        t = self.expr_type(ex, strict=False)
                        if t:
                            self.vars.setdefault(nm, t)

    def expr_type(self, ex: str, strict: bool = True):
        """Go type of an argument expression (the forms the shim uses), or None (strict: raise)."""
        ex = ex.strip()
        m = re.fullmatch(r"\(\*C\.(\w+)\)\((.*)\)", ex, re.S)
        if m:
            return f"*C.{m.group(1)}"
        m = re.fullmatch(r"C\.(\w+)\((.*)\)", ex, re.S)
        if m:
            if m.group(1).startswith("nsx_"):
                ret = header_prototypes()[m.group(1)][0]
                return "C." + ret if not ret.endswith("*") else "*C." + ret[:-1]
            return f"C.{m.group(1)}"
        if ex.startswith("&"):
            inner = self.expr_type(ex[1:], strict)
            return None if inner is None else "*" + inner
        m = re.fullmatch(r"(\w+)\((.*)\)", ex, re.S)
        if m and m.group(1) in self.funcs:
            return self.funcs[m.group(1)]
        if re.fullmatch(r"\w+", ex) and ex in self.vars:
            return self.vars[ex]
        m = re.fullmatch(r"\w+\.(\w+)", ex)
        if m and m.group(1) in self.fields:
            return self.fields[m.group(1)]
        if strict:
            raise AssertionError(f"{os.path.basename(self.path)}: cannot type argument {ex!r}")
        return None

    def c_calls(self) -> list:
        """[(function, [argument expressions])] for every C.nsx_* call."""
        calls = []
        for m in re.finditer(r"\bC\.(nsx_\w+)\(", self.src):
            i = m.end() - 1
            calls.append((m.group(1), _split_args(self.src[i + 1:_close(self.src, i)])))
        return calls


@pytest.fixture(scope="module")
def shim():
    return [GoFile(os.path.join(GO_DIR, f)) for f in SHIM_FILES]


def test_every_c_call_matches_the_header(shim):
    protos = header_prototypes()
    exported = set(re.findall(r" T (nsx_\w+)", subprocess.run(
        ["nm", "-D", "--defined-only", nsx.LIB_PATH], capture_output=True, text=True).stdout))
    seen = set()
    for gf in shim:
        calls = gf.c_calls()
        assert calls, gf.path
        for fn, args in calls:
            where = f"{os.path.basename(gf.path)}: C.{fn}"
            assert fn in protos, f"{where} is not declared in include/nsx_csum.h"
            assert fn in exported, f"{where} is not exported by libnsx_csum.so"
            _, params = protos[fn]
            assert len(args) == len(params), f"{where}: {len(args)} arguments, the header declares {len(params)}"
            for k, (a, want) in enumerate(zip(args, params)):
                got = go_to_c(gf.expr_type(a))
                assert got == want, f"{where} argument {k} {a!r}: cgo would pass {got}, the header takes {want}"
            seen.add(fn)
    # the shim's surface: single-segment host sum, pinned staging, the host batch and receive passes
    assert seen >= {"nsx_csum16", "nsx_strerror", "nsx_alloc_pinned", "nsx_free_pinned", "nsx_csum_ragged_host",
                    "nsx_rx_ipv4_tcp_verify_host", "nsx_rx_ipv6_tcp_verify_host", "nsx_tcp_build_host",
                    "nsx_tcp_wire_len"}, seen


def test_struct_fields_the_shim_sets_exist(shim):
    """Every `h.<field> = (*C.<type>)(...)` the sender shim writes into a C struct names a member the header's
    struct declares, with the member's type (const stripped) — what cgo checks for struct field assignments."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    members = {}
    for body, name in re.findall(r"typedef\s+struct\s*\{([^}]*)\}\s*(\w+)\s*;", src):
        for t, m in re.findall(r"((?:const\s+)?\w+\s*\*?)\s*(\w+)\s*;", body):
            members[(name, m)] = _norm(t)
    checked = 0
    for gf in shim:
        for var, typ in gf.vars.items():
            tm = re.fullmatch(r"C\.(\w+)", typ)
            if not tm or tm.group(1) not in header_typedefs():
                continue
            for fld, rhs in re.findall(rf"\b{var}\.(\w+)\s*=\s*([^\n]+)", gf.src):
                assert (tm.group(1), fld) in members, f"{gf.path}: {tm.group(1)} has no member {fld}"
                assert go_to_c(gf.expr_type(rhs)) == members[(tm.group(1), fld)], (gf.path, fld, rhs)
                checked += 1
    assert checked == 8  # build_nsx.go fills all eight nsx_tcp_hdr_soa members


def test_constants_types_and_preamble(shim):
    consts = header_constants()
    protos = header_prototypes()
    for gf in shim:
        for c in set(re.findall(r"\bC\.(NSX_\w+)", gf.src)):
            assert c in consts, f"{gf.path}: C.{c} is not #defined in include/nsx_csum.h"
        for t in set(re.findall(r"\bC\.(\w+)", gf.src)) - {c for c in consts} - set(protos) - {"GoString"}:
            assert t in ("uint8_t", "uint16_t", "uint32_t", "uint64_t", "size_t", "int") or t in header_typedefs(), \
                (gf.path, t)
        assert '#include "nsx_csum.h"' in open(gf.path).read(), gf.path
        assert open(gf.path).read().startswith("//go:build nsx"), gf.path
    assert "#cgo LDFLAGS: -lnsx_csum" in open(os.path.join(GO_DIR, "checksum_nsx.go")).read()


def test_the_shim_calls_compile_and_link_as_c(shim, tmp_path):
    """The calls rebuilt as C with the argument types cgo passes (locals of exactly those types), compiled
    -Wall -Werror against the header and linked against the library (never run: the body is unreachable)."""
    body = []
    for gf in shim:
        for fn, args in gf.c_calls():
            decls = "".join(f"{go_to_c(gf.expr_type(a))} a{k} = 0; " for k, a in enumerate(args))
            body.append(f"    {{ {decls}(void){fn}({', '.join(f'a{k}' for k in range(len(args)))}); }}")
    src = tmp_path / "shim_calls.c"
    src.write_text("#include \"nsx_csum.h\"\nint main(int argc, char** argv) {\n    (void)argv;\n"
                   "    if (argc < 1000) return 0;\n" + "\n".join(body) + "\n    return 1;\n}\n")
    exe = tmp_path / "shim_calls"
    libdir = os.path.dirname(nsx.LIB_PATH)
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-Wno-unused-variable", str(src), "-I",
                        os.path.join(ROOT, "include"), "-L", libdir, "-lnsx_csum", f"-Wl,-rpath,{libdir}",
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr + src.read_text()
    assert subprocess.run([str(exe)]).returncode == 0


def test_checker_catches_a_mismatch():
    """The type inference is strict: an argument of the wrong C type or a wrong count is reported."""
    gf = GoFile.__new__(GoFile)
    gf.path, gf.vars, gf.funcs, gf.fields = "x.go", {"partial": "*C.uint16_t"}, {}, {}
    assert go_to_c(gf.expr_type("partial")) == "uint16_t*" != header_prototypes()["nsx_csum_ragged_host"][1][3]
    assert go_to_c(gf.expr_type("C.int(n)")) == "int" != header_prototypes()["nsx_csum_ragged_host"][1][2]
    with pytest.raises(AssertionError):
        gf.expr_type("someUntypedThing")


def _go_funcs(src: str) -> dict:
    """name (receiver type prefixed: 'PinnedBatch.Verify') -> body text, for every func in a Go source."""
    out = {}
    for m in re.finditer(r"^func\s+(?:\(\s*\w+\s+\*?(\w+)\s*\)\s*)?(\w+)(?:\[[^\]]*\])?\s*\(", src, re.M):
        i = src.index("{", _close(src, m.end() - 1))
        depth = 0
        for j in range(i, len(src)):
            depth += {"{": 1, "}": -1}.get(src[j], 0)
            if depth == 0:
                break
        out[(m.group(1) + "." if m.group(1) else "") + m.group(2)] = src[i:j + 1]
    return out


def test_go_entry_points_pin_memory_only_when_a_batch_outgrows_the_block(shim):
    """the Go side must not pin (hipHostMalloc) and unpin per call — page registration costs
    milliseconds against a small batch's tens of microseconds. Checked on the shim's source:
      - nsx_alloc_pinned is called in exactly one place, pinnedArena.reserve, after its early return for a block
        that is already large enough (grow-only, at least doubling), and nsx_free_pinned only in pinnedArena.free;
      - the reuse forms a transport keeps across batches — PinnedBatch.Checksum, PinnedBatch.Verify (rx),
        Sender.Build — reach the library with no allocation or free of pinned memory of their own;
      - the one-shot forms (ChecksumSegments, VerifyDatagrams/VerifyPackets6, BuildSegments) are wrappers over
        them."""
    funcs = {}
    for gf in shim:
        funcs.update(_go_funcs(gf.src))
    where_alloc = [k for k, b in funcs.items() if "C.nsx_alloc_pinned" in b]
    where_free = [k for k, b in funcs.items() if "C.nsx_free_pinned" in b]
    assert where_alloc == ["pinnedArena.reserve"], where_alloc
    assert where_free == ["pinnedArena.free"], where_free
    res = funcs["pinnedArena.reserve"]
    assert re.search(r"if n <= uint64\(len\(a\.buf\)\) \{\s*return nil", res)
    assert res.index("return nil") < res.index("C.nsx_alloc_pinned") and "c *= 2" in res
    for k, call in (("PinnedBatch.Checksum", "C.nsx_csum_ragged_host"), ("PinnedBatch.Verify", "C.nsx_rx_ipv4_tcp_verify_host"),
                    ("PinnedBatch.Verify", "C.nsx_rx_ipv6_tcp_verify_host"), ("build", "C.nsx_tcp_build_host")):
        assert call in funcs[k], (k, call)
        assert "NewPinnedBatch" not in funcs[k] and ".free()" not in funcs[k] and ".Free()" not in funcs[k], k
    assert "build(&s.arena" in funcs["Sender.Build"] and "arena.reserve(" in funcs["build"]
    assert "b.Checksum(" in funcs["ChecksumSegments"] and "b.Verify(" in funcs["verifyFrames"]
    assert "verifyFrames(" in funcs["VerifyDatagrams"] and "verifyFrames(" in funcs["VerifyPackets6"]
    assert "build(a, b" in funcs["BuildSegments"]
    # the sender's C call sees only pinned memory: every pointer argument is a region of the arena
    gf = next(g for g in shim if g.path.endswith("build_nsx.go"))
    (fn, args), = [c for c in gf.c_calls() if c[0] == "nsx_tcp_build_host"]
    for a in args:
        assert a.startswith(("&h", "(*C.uint8_t)(region(", "(*C.uint64_t)(region(", "(*C.uint16_t)(region(",
                             "optOffs", "partial", "C.uint64_t(n)", "C.int(")), a
