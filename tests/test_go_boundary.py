"""Drift guard for the Go boundary (go/**/*.go -> include/deoss_merkle.h), CPU only.

There is no Go toolchain in this image, so the cgo packages are never
type-checked.  This test does the part of that check that matters for the C ABI: every
`C.dm_*(...)` call in the Go sources names a function the header declares, passes exactly as many
arguments as its prototype takes, and passes a pointer where the prototype has a pointer (or an
array) and an integer where it has an integer; every `C.DM_*` constant exists in the header.
The contract the Go packages keep is /root/reference/common/hashtree/types.go:19
(NewHashTree(chunkPath []string) (*merkletree.MerkleTree, error)); this guards what is under it.
"""
import glob
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "deoss_merkle.h")
INT_CASTS = ("C.uint64_t(", "C.int(", "C.uint32_t(", "C.int64_t(", "C.size_t(", "C.double(", "C.uint8_t(",
             "C.uint(", "C.long(", "C.ulong(", "C.char(")


def _strip_c_comments(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", " ", text)


RETURNS = {}   # dm_* function -> kind of its result ('ptr' / 'int' / 'void'), filled by header_api


def header_api(path=HEADER):
    """(prototypes {name: [kind, ...]}, constants {name}) of the C header; kind 'ptr' or 'int'."""
    text = _strip_c_comments(open(path).read())
    protos = {}
    for m in re.finditer(r"\b(int|void|uint64_t|uint32_t|const\s+char\s*\*)\s*(\**)\s*(dm_\w+)\s*\(([^;{]*?)\)\s*;",
                         text, flags=re.S):
        params = [p.strip() for p in m.group(4).split(",")]
        if params == ["void"] or params == [""]:
            params = []
        protos[m.group(3)] = ["ptr" if ("*" in p or "[" in p) else "int" for p in params]
        ret = m.group(1)
        RETURNS[m.group(3)] = "ptr" if ("*" in ret or m.group(2)) else ("void" if ret == "void" else "int")
    consts = set(re.findall(r"\b(DM_[A-Z0-9_]+)\s*=", text)) | set(re.findall(r"#define\s+(DM_[A-Z0-9_]+)", text))
    return protos, consts


def _strip_go_comments(src):
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if c in "\"'`":
            q = c
            j = i + 1
            while j < n and src[j] != q:
                j += 2 if (src[j] == "\\" and q != "`") else 1
            out.append(src[i:j + 1])
            i = j + 1
        elif src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            i = n if j < 0 else j + 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


def _split_args(s):
    args, depth, cur = [], 0, []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            args.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    last = "".join(cur).strip()
    if last:
        args.append(last)
    return args


def go_calls(src):
    """[(name, [arg text, ...], line)] of every C.dm_* call in Go source (comments removed)."""
    code = _strip_go_comments(src)
    calls = []
    for m in re.finditer(r"\bC\.(dm_\w+)\s*\(", code):
        i, depth = m.end(), 1
        j = i
        while j < len(code) and depth:
            if code[j] == "(":
                depth += 1
            elif code[j] == ")":
                depth -= 1
            j += 1
        calls.append((m.group(1), _split_args(code[i:j - 1]), code.count("\n", 0, m.start()) + 1))
    return calls, code


def _decl_kind(name, code, seen):
    """Kind of identifier `name` from its declaration in the same file (params, fields, var, :=)."""
    if name in seen:
        return None
    seen = seen | {name}
    n = re.escape(name)
    if re.search(rf"\b{n}\s+\*+C\.\w+", code) or re.search(rf"\b{n}\s+\[\]\*C\.", code) or \
            re.search(rf"\b{n}\s+unsafe\.Pointer\b", code):
        return "ptr"
    if re.search(rf"\b{n}\s+C\.(?:u?int\w*|size_t|double|char|long|ulong)\b", code):
        return "int"
    for m in re.finditer(rf"(?:^|[\s(,])(?:var\s+)?{n}\s*(?:,\s*\w+\s*)*:?=\s*([^\n]+)", code):
        k = arg_kind(m.group(1).strip(), code, seen)
        if k:
            return k
    return None


def arg_kind(a, code, seen=frozenset()):
    a = a.strip()
    if a == "nil" or a.startswith("&") or a.startswith("unsafe.Pointer(") or a.startswith("C.CString(") \
            or re.match(r"^\(\*+[\w.]+\)\(", a) or re.match(r"^\(\*+unsafe\.Pointer\)\(", a):
        return "ptr"
    if a.startswith(INT_CASTS) or re.match(r"^-?\d+$", a) or re.match(r"^C\.DM_\w+$", a):
        return "int"
    m = re.match(r"^C\.(dm_\w+)\(", a)              # result of another C call
    if m:
        return RETURNS.get(m.group(1))
    m = re.match(r"^([A-Za-z_]\w*)\(.*\)$", a, flags=re.S)   # result of a Go function of the package
    if m:
        f = re.escape(m.group(1))
        if re.search(rf"\bfunc\s+{f}\s*\([^)]*\)\s*\(?\s*\*C\.", code):
            return "ptr"
        if re.search(rf"\bfunc\s+{f}\s*\([^)]*\)\s*\(?\s*C\.(?:u?int\w*|size_t)\b", code):
            return "int"
        return None
    m = re.match(r"^([\w.]+)\[.*\]$", a)           # element of a slice of C pointers
    if m:
        sl = re.escape(m.group(1).split(".")[-1])
        if re.search(rf"\b{sl}\s*(?::?=\s*make\(\s*)?\[\]\*C\.", code):
            return "ptr"
        return None
    m = re.match(r"^<-\s*([\w.]+)$", a)           # receive from a channel of C pointers
    if m:
        ch = re.escape(m.group(1).split(".")[-1])
        if re.search(rf"\b{ch}\s*(?:=\s*make\(\s*)?chan\s+\*C\.", code):
            return "ptr"
        return None
    m = re.match(r"^([A-Za-z_]\w*)(?:\.([A-Za-z_]\w*))*$", a)
    if m:
        return _decl_kind(a.split(".")[-1], code, seen)
    return None


def check_go(src, protos, consts, where="<src>", package_code=""):
    """Problems of one Go source against the header (empty list = consistent).  package_code: the
    other files of the same Go package (declarations an argument may refer to)."""
    problems = []
    calls, code = go_calls(src)
    code = code + "\n" + _strip_go_comments(package_code)
    for name, args, line in calls:
        if name not in protos:
            problems.append(f"{where}:{line}: C.{name} is not declared in include/deoss_merkle.h")
            continue
        want = protos[name]
        if len(args) != len(want):
            problems.append(f"{where}:{line}: C.{name} takes {len(want)} arguments, the call passes {len(args)}")
            continue
        for i, (a, k) in enumerate(zip(args, want)):
            got = arg_kind(a, code)
            if got is None:
                problems.append(f"{where}:{line}: C.{name} argument {i + 1} ({a!r}): kind not determined")
            elif got != k:
                problems.append(f"{where}:{line}: C.{name} argument {i + 1} ({a!r}) is {got}, the prototype wants {k}")
    for c in sorted(set(re.findall(r"\bC\.(DM_[A-Z0-9_]+)\b", code))):
        if c not in consts:
            problems.append(f"{where}: C.{c} is not defined in include/deoss_merkle.h")
    return problems, len(calls)


def go_sources():
    return sorted(glob.glob(os.path.join(ROOT, "go", "**", "*.go"), recursive=True))


def test_every_go_call_matches_the_header():
    protos, consts = header_api()
    assert len(protos) > 60 and "dm_new_hash_tree" in protos and protos["dm_root_buffer"] == \
        ["ptr", "ptr", "int", "int", "ptr", "ptr"]
    total, problems = 0, []
    for path in go_sources():
        pkg = "\n".join(open(q).read() for q in go_sources() if os.path.dirname(q) == os.path.dirname(path)
                        and q != path)
        p, n = check_go(open(path).read(), protos, consts, os.path.relpath(path, ROOT), pkg)
        problems += p
        total += n
    assert total >= 50, total                  # every binding file was scanned
    assert problems == [], "\n".join(problems)


def test_go_binds_the_header_it_checks_against():
    """Every file calling C.dm_* includes the header this test parses, and every package links it
    through pkg-config (#cgo flags of one file apply to its whole package)."""
    pkgs = {}
    for path in go_sources():
        src = open(path).read()
        if "C.dm_" in src:
            assert '#include "deoss_merkle.h"' in src or "#include <deoss_merkle.h>" in src, path
            pkgs.setdefault(os.path.dirname(path), []).append(src)
    assert len(pkgs) == 3
    for d, srcs in pkgs.items():
        assert any("#cgo pkg-config: deoss_merkle" in x for x in srcs), d


def test_guard_catches_a_mismatched_call():
    """The guard fails on deliberately wrong calls: a missing argument, an integer where the
    prototype has a pointer, an unknown function and an unknown constant."""
    protos, consts = header_api()
    bad = """package x
// #include "deoss_merkle.h"
import "C"
import "unsafe"
func f(c *C.dm_ctx, buf []byte) {
	var root [32]byte
	C.dm_root_buffer(c, unsafe.Pointer(&buf[0]), C.uint64_t(len(buf)), nil, (*C.uint8_t)(&root[0]))
	C.dm_root_buffer(c, C.uint64_t(len(buf)), C.uint64_t(len(buf)), C.uint64_t(1), nil, (*C.uint8_t)(&root[0]))
	C.dm_no_such_call(c)
	_ = C.DM_ERR_NOPE
}
"""
    problems, n = check_go(bad, protos, consts)
    assert n == 3
    text = "\n".join(problems)
    assert "takes 6 arguments, the call passes 5" in text
    assert "argument 2 ('C.uint64_t(len(buf))') is int, the prototype wants ptr" in text
    assert "C.dm_no_such_call is not declared" in text
    assert "C.DM_ERR_NOPE is not defined" in text
    good = bad.replace("C.dm_no_such_call(c)\n", "").replace("_ = C.DM_ERR_NOPE\n", "")
    good = good.replace("C.dm_root_buffer(c, C.uint64_t(len(buf)), C.uint64_t(len(buf)),",
                        "C.dm_root_buffer(c, unsafe.Pointer(&buf[0]), C.uint64_t(len(buf)),")
    good = good.replace("C.uint64_t(len(buf)), nil, (*C.uint8_t)(&root[0]))\n\tC.dm_root_buffer(c, unsafe",
                        "C.uint64_t(len(buf)), C.uint64_t(1), nil, (*C.uint8_t)(&root[0]))\n\tC.dm_root_buffer(c, unsafe")
    assert check_go(good, protos, consts)[0] == []


# ---- the C side of cgo, compiled -----------------------------------------
# Go cannot compile here, but cgo's C half can: every Go file's preamble (the comment right above
# `import "C"`) is C that cgo hands to the C compiler with the package's `#cgo pkg-config` flags,
# and the package then links the library those flags name.

def cgo_preambles():
    """[(path, preamble C text without #cgo lines)] of every Go file that imports "C"."""
    out = []
    for path in go_sources():
        src = open(path).read()
        m = re.search(r"/\*((?:(?!\*/).)*)\*/\s*\nimport \"C\"", src, flags=re.S)
        if m is None:
            m2 = re.search(r"((?:^//[^\n]*\n)+)import \"C\"", src, flags=re.M)
            if m2 is None:
                assert 'import "C"' not in src, f"{path}: import \"C\" without a preamble this test can read"
                continue
            text = "\n".join(ln[2:] for ln in m2.group(1).splitlines())
        else:
            text = m.group(1)
        out.append((path, "\n".join(ln for ln in text.splitlines() if not ln.strip().startswith("#cgo"))))
    return out


def pkg_config(pc_path):
    """(cflags, libs) of a .pc file, expanded the way pkg-config does (${var} substitution).  This
    image has no pkg-config binary; cgo's `#cgo pkg-config: deoss_merkle` runs the real one."""
    vars_, fields = {}, {}
    for line in open(pc_path):
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        if "=" in line and ":" not in line.split("=")[0]:
            k, v = line.split("=", 1)
            vars_[k.strip()] = v.strip()
        elif ":" in line:
            k, v = line.split(":", 1)
            fields[k.strip()] = v.strip()

    def expand(v):
        for _ in range(8):
            for k, x in vars_.items():
                v = v.replace("${" + k + "}", x)
        assert "${" not in v, v
        return v.split()
    return expand(fields.get("Cflags", "")), expand(fields.get("Libs", ""))


def _built_pc():
    from deoss_amd import build as b
    b.build(verbose=False)
    return os.path.join(ROOT, "deoss_amd", "deoss_merkle.pc")


def test_every_cgo_preamble_compiles_as_c99(tmp_path):
    """Each preamble + the header compiles with gcc -std=c99 -pedantic -Werror -Wall -Wextra and
    the package's pkg-config cflags: what cgo compiles first when `go build -tags hip` runs."""
    cflags, _ = pkg_config(_built_pc())
    pre = cgo_preambles()
    importing = [q for q in go_sources() if 'import "C"' in open(q).read()]
    assert len(pre) == len(importing) >= 7 and all('#include "deoss_merkle.h"' in p for _, p in pre)
    for i, (path, text) in enumerate(pre):
        src = tmp_path / f"preamble_{i}.c"
        src.write_text(text + "\nint deoss_cgo_preamble_unit;\n")
        r = subprocess.run(["gcc", "-std=c99", "-pedantic", "-Werror", "-Wall", "-Wextra", *cflags, "-c", str(src),
                            "-o", str(tmp_path / f"preamble_{i}.o")], capture_output=True, text=True)
        assert r.returncode == 0, (os.path.relpath(path, ROOT), r.stderr)


def test_c_program_links_through_the_pc_file(tmp_path):
    """A C program built with only the .pc file's flags (as cgo links go/hashtree) loads the library
    and gets the reference's empty-list error text (/root/reference/common/hashtree/types.go:20-22)
    from dm_strerror; without a GPU dm_create returns DM_ERR_NODEV and no context, with one it
    succeeds."""
    cflags, libs = pkg_config(_built_pc())
    src = tmp_path / "cgo_link.c"
    src.write_text(r'''
#include <stdio.h>
#include <string.h>
#include "deoss_merkle.h"
int main(void) {
    dm_ctx *c = NULL;
    int rc, gpus;
    if (strcmp(dm_strerror(DM_ERR_EMPTY), "Empty data") != 0) return 10;
    gpus = dm_gpu_count();
    rc = dm_create(&c, NULL, 0);
    printf("%d %d %d\n", gpus, rc, c != NULL);
    if (c) dm_destroy(c);
    return 0;
}
''')
    exe = tmp_path / "cgo_link"
    r = subprocess.run(["gcc", "-std=c99", "-pedantic", "-Werror", "-Wall", *cflags, str(src), "-o", str(exe), *libs],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    gpus, rc, have = map(int, r.stdout.split())
    if gpus == 0:
        assert (rc, have) == (-7, 0)          # DM_ERR_NODEV, no context: no silent CPU fallback
    else:
        assert (rc, have) == (0, 1)
