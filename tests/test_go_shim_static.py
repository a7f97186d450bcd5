"""Static checks of the Go shim (go/gpueval) against the C-ABI headers.

The image has no Go toolchain, so the cgo binding is never compiled here.  These checks read the Go
sources as text and hold every cgo reference to what the headers its preamble includes declare:
  * every `C.name` a file uses is declared by its own preamble's headers (cgo resolves each file's
    names through that file's preamble only), or is a cgo builtin / a libc function of an included
    system header;
  * every call of a `kgpu_*` entry point passes as many arguments as the prototype declares;
  * every snake_case field selected on a value (`x.n_terms`) is a field of some header struct.
No GPU, no Go: a CPU test of the shipped drop-in's binding surface (include/kgpu.h, include/kgpu_compile.h).
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "gpueval")
INC = os.path.join(ROOT, "include")
if not os.path.isdir(GO):  # the GPU box's copy of the tree leaves go/ out (.gpurunignore): CPU-only checks
    pytest.skip("go/gpueval is not in this copy of the tree", allow_module_level=True)

CGO_BUILTINS = {"CString", "GoString", "GoStringN", "GoBytes", "CBytes"}
C_SCALARS = {"char", "schar", "uchar", "short", "ushort", "int", "uint", "long", "ulong", "longlong", "ulonglong",
             "float", "double", "size_t", "int8_t", "int16_t", "int32_t", "int64_t", "uint8_t", "uint16_t",
             "uint32_t", "uint64_t", "uintptr_t"}
LIBC = {"stdlib.h": {"free", "malloc", "calloc", "realloc"}, "string.h": {"memcpy", "memset", "strlen", "memcmp"}}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _header(name, seen):
    """Declarations of header `name` (include/) and of the project headers it includes."""
    path = os.path.join(INC, name)
    if name in seen or not os.path.exists(path):
        return ""
    seen.add(name)
    text = _strip_c_comments(open(path).read())
    out = [text]
    for inc in re.findall(r'#include\s+"([^"]+)"', text):
        out.append(_header(inc, seen))
    return "\n".join(out)


def _split_args(s):
    """Top-level comma split of a Go argument list (strings, runes and brackets respected)."""
    args, depth, cur, i = [], 0, [], 0
    while i < len(s):
        ch = s[i]
        if ch in "\"'`":
            j = i + 1
            while j < len(s) and s[j] != ch:
                j += 2 if (s[j] == "\\" and ch != "`") else 1
            cur.append(s[i:j + 1])
            i = j + 1
            continue
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            args.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
        i += 1
    tail = "".join(cur).strip()
    if tail or args:
        args.append(tail)
    return [a for a in (x.strip() for x in args) if a]


def _call_args(src, start):
    """The argument text of the call whose '(' is at src[start]."""
    depth, i = 0, start
    while i < len(src):
        ch = src[i]
        if ch in "\"'`":
            j = i + 1
            while j < len(src) and src[j] != ch:
                j += 2 if (src[j] == "\\" and ch != "`") else 1
            i = j + 1
            continue
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
            if depth == 0:
                return src[start + 1:i]
        i += 1
    raise AssertionError("unbalanced call at offset %d" % start)


class Decls:
    def __init__(self, text):
        self.text = text
        self.protos = {}
        for m in re.finditer(r"\b(kgpu_\w+)\s*\(([^;{]*?)\)\s*;", text):
            params = [p for p in (x.strip() for x in m.group(2).split(",")) if p]
            if params == ["void"]:
                params = []
            self.protos[m.group(1)] = len(params)
        self.names = set(re.findall(r"#define\s+(\w+)", text))
        self.names |= set(re.findall(r"\}\s*(\w+)\s*;", text))              # typedef struct {...} name;
        self.names |= set(re.findall(r"typedef\s+[\w\s\*]+?\b(\w+)\s*;", text))  # typedef struct x x; / scalars
        self.names |= set(re.findall(r"\benum\s*\w*\s*\{([^}]*)\}", text) and
                          [n for body in re.findall(r"\benum\s*\w*\s*\{([^}]*)\}", text)
                           for n in re.findall(r"\b([A-Z][A-Z0-9_]+)\s*(?:=|,|$)", body)])
        self.names |= set(self.protos)
        self.fields = set()
        for body in re.findall(r"struct\s*\w*\s*\{([^}]*)\}", text):
            for decl in body.split(";"):
                decl = re.sub(r"\[[^\]]*\]", "", decl).strip()
                if not decl:
                    continue
                for part in decl.split(","):
                    m = re.search(r"(\w+)\s*$", part.strip())
                    if m:
                        self.fields.add(m.group(1))


def _go_files():
    return sorted(f for f in os.listdir(GO) if f.endswith(".go"))


def _preamble(src):
    m = re.search(r"/\*(.*?)\*/\s*import\s+\"C\"", src, flags=re.S)
    if m:
        return m.group(1)
    lines = []
    for ln in src.splitlines():
        if ln.startswith("// "):
            lines.append(ln[3:])
        elif ln.startswith('import "C"'):
            return "\n".join(lines)
        else:
            lines = []
    return ""


def _strip_go(src):
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


FILES = [f for f in _go_files() if 'import "C"' in open(os.path.join(GO, f)).read()]
ALL_DECLS = Decls(_header("kgpu.h", set()) + "\n" + _header("kgpu_compile.h", set()))


def test_go_sources_present():
    assert FILES, "no cgo files under go/gpueval"
    assert {"kgpu.go", "compile.go", "desc.go", "plugin.go"} <= set(_go_files())


@pytest.mark.parametrize("fname", FILES)
def test_cgo_names_declared_by_the_files_preamble(fname):
    raw = open(os.path.join(GO, fname)).read()
    pre = _preamble(raw)
    seen = set()
    decl_text = "\n".join(_header(h, seen) for h in re.findall(r'#include\s+"([^"]+)"', pre))
    decl_text += "\n" + _strip_c_comments(pre)  # names the preamble defines itself
    d = Decls(decl_text)
    libc = set()
    for h in re.findall(r"#include\s+<([^>]+)>", pre):
        libc |= LIBC.get(h, set())
    src = _strip_go(raw)
    missing = sorted({n for n in re.findall(r"\bC\.([A-Za-z_]\w*)", src)
                      if n not in CGO_BUILTINS and n not in C_SCALARS and n not in libc and n not in d.names
                      and not n.startswith("struct_")})
    assert not missing, "%s uses C names its preamble does not declare: %s" % (fname, missing)


@pytest.mark.parametrize("fname", FILES)
def test_entry_point_arity(fname):
    src = _strip_go(open(os.path.join(GO, fname)).read())
    bad = []
    n_calls = 0
    for m in re.finditer(r"\bC\.(kgpu_\w+)\s*\(", src):
        name = m.group(1)
        if name not in ALL_DECLS.protos:
            continue  # a type conversion, e.g. C.kgpu_str(x)
        n_calls += 1
        args = _split_args(_call_args(src, m.end() - 1))
        if len(args) != ALL_DECLS.protos[name]:
            bad.append("%s: %d args, prototype %d" % (name, len(args), ALL_DECLS.protos[name]))
    assert not bad, "%s: %s" % (fname, bad)


def test_every_go_entry_point_call_is_counted():
    total = 0
    for f in FILES:
        src = _strip_go(open(os.path.join(GO, f)).read())
        total += sum(1 for m in re.finditer(r"\bC\.(kgpu_\w+)\s*\(", src) if m.group(1) in ALL_DECLS.protos)
    assert total >= 40, total  # the binding calls most of the ABI (kgpu.go, compile.go, ...)


@pytest.mark.parametrize("fname", FILES)
def test_snake_case_fields_exist_in_header_structs(fname):
    src = _strip_go(open(os.path.join(GO, fname)).read())
    src = re.sub(r'"(\\.|[^"\\])*"|`[^`]*`', '""', src)  # string literals
    used = set(re.findall(r"(?<!\bC)\.([a-z][a-z0-9]*_[a-z0-9_]+)\b", src))
    # composite literal keys of C structs: C.kgpu_x{a_b: ...}
    for body in re.findall(r"\bC\.kgpu_\w+\{([^{}]*)\}", src):
        used |= set(re.findall(r"\b([a-z][a-z0-9_]*)\s*:", body))
    missing = sorted(u for u in used if u not in ALL_DECLS.fields)
    assert not missing, "%s selects fields no header struct has: %s" % (fname, missing)


def test_no_duplicate_package_level_declarations():
    """One package: a function, method (per receiver type), type, var or const declared twice is a compile error."""
    seen, dup = {}, []
    for f in _go_files():
        src = _strip_go(open(os.path.join(GO, f)).read())
        names = []
        for m in re.finditer(r"^func\s+(?:\(\s*\w*\s*\*?\s*(\w+)\s*\)\s*)?(\w+)\s*\(", src, flags=re.M):
            names.append((m.group(1) or "", m.group(2)))
        names += [("", n) for n in re.findall(r"^type\s+(\w+)\s", src, flags=re.M)]
        names += [("", n) for n in re.findall(r"^(?:var|const)\s+(\w+)\s", src, flags=re.M)]
        for block in re.findall(r"^(?:var|const|type)\s*\(\n(.*?)^\)", src, flags=re.M | re.S):
            names += [("", n) for n in re.findall(r"^\s*(\w+)\b", block, flags=re.M)]
        for key in names:
            if key[1] in ("_", "init"):
                continue
            if key in seen and seen[key] != f or key in seen and names.count(key) > 1:
                dup.append("%s (%s, %s)" % (".".join(k for k in key if k), seen[key], f))
            seen.setdefault(key, f)
    assert not dup, dup


@pytest.mark.parametrize("fname", _go_files())
def test_every_import_is_used(fname):
    """An imported package no code of the file names is a Go compile error."""
    src = _strip_go(open(os.path.join(GO, fname)).read())
    imports = []
    for block in re.findall(r"^import\s*\((.*?)\)", src, flags=re.M | re.S):
        imports += re.findall(r"^\s*(\w+\s+)?\"([^\"]+)\"", block, flags=re.M)
    imports += re.findall(r"^import\s+(\w+\s+)?\"([^\"]+)\"", src, flags=re.M)
    body = re.sub(r"^import\s*\(.*?\)", "", src, flags=re.M | re.S)
    body = re.sub(r"^import\s+[^\n]*", "", body, flags=re.M)
    unused = []
    for alias, path in imports:
        name = alias.strip() if alias else path.rsplit("/", 1)[-1]
        if path == "C" or name in ("_", "."):
            continue
        if not re.search(r"\b%s\." % re.escape(name), body):
            unused.append(path)
    assert not unused, "%s imports packages it never names: %s" % (fname, unused)


GO_BUILTINS = {"len", "cap", "append", "make", "new", "copy", "delete", "panic", "recover", "print", "println",
               "close", "complex", "real", "imag"}  # go 1.13: no min / max / clear


def _package_names():
    funcs, methods, fields, types = set(), set(), set(), set()
    for f in _go_files():
        src = _strip_go(open(os.path.join(GO, f)).read())
        for m in re.finditer(r"^func\s+(\(\s*\w*\s*\*?\s*\w+\s*\)\s*)?(\w+)\s*\(", src, flags=re.M):
            (methods if m.group(1) else funcs).add(m.group(2))
        types |= set(re.findall(r"^type\s+(\w+)\s", src, flags=re.M))
        for body in re.findall(r"\bstruct\s*\{(.*?)^\}", src, flags=re.M | re.S):
            fields |= set(re.findall(r"^\s*(\w+)\s+func\b", body, flags=re.M))
    return funcs, methods, fields, types


def test_unexported_calls_resolve_in_the_package():
    """A call of an unexported name -- x.name(...) or name(...) -- must resolve to this package's methods,
    functions or func-typed fields, a local closure, or a go 1.13 builtin (no min / max)."""
    funcs, methods, fields, types = _package_names()
    bad = []
    for f in _go_files():
        src = _strip_go(open(os.path.join(GO, f)).read())
        src = re.sub(r'"(\\.|[^"\\])*"|`[^`]*`', '""', src)
        # local closures and func-typed variables / parameters: name := func / name = func / name func(
        local = set(re.findall(r"\b(\w+)\s*:?=\s*func\b", src)) | set(re.findall(r"\b(\w+)\s+func\s*\(", src))
        for m in re.finditer(r"(\bC\.|\.)?\b([a-z]\w*)\s*\(", src):
            sel, name = m.group(1), m.group(2)
            if sel == "C.":
                continue  # cgo: checked against the headers above
            if name in ("func", "if", "for", "switch", "return", "go", "defer", "range", "select", "case", "interface",
                        "struct", "map", "chan", "type", "var", "const", "import"):
                continue
            if sel:
                if name not in methods and name not in fields and name not in local:
                    bad.append("%s: .%s(" % (f, name))
            else:
                pre = src[max(0, m.start() - 6):m.start()]
                if re.search(r"func\s*$", pre) or re.search(r"\)\s*$", pre):
                    continue  # a declaration, or a method value / type conversion context
                if name not in GO_BUILTINS and name not in funcs and name not in local and name not in types \
                        and name not in methods and not re.match(r"^(u?int(8|16|32|64)?|float(32|64)|byte|rune|string|"
                                                                 r"bool|uintptr|error)$", name):
                    bad.append("%s: %s(" % (f, name))
    assert not bad, sorted(set(bad))


# APIs newer than the reference module's go 1.13 (go.mod `go 1.13`)
POST_113 = [r"\bunsafe\.(Slice|String|StringData|SliceData|Add)\b", r"\bany\b", r"\bstrings\.(Cut|Clone|CutPrefix)\b",
            r"\bbytes\.Cut\b", r"\bos\.(ReadFile|WriteFile|ReadDir)\b", r"\bio\.(ReadAll|Discard|NopCloser)\b",
            r"\bmath\.(MaxInt|MinInt|MaxUint)\b", r"\batomic\.(Int32|Int64|Uint32|Uint64|Bool|Pointer|Value)\b\s*[{)]",
            r"\bfunc\s+\w+\s*\[", r"\btype\s+\w+\s*\[\s*\w+\s+(any|comparable|interface)", r"\bslices\.", r"\bmaps\.",
            r"\berrors\.Join\b", r"\bcontext\.(WithoutCancel|AfterFunc|Cause)\b", r"\bsync\.OnceValue"]


@pytest.mark.parametrize("fname", _go_files())
def test_go_113_only(fname):
    src = _strip_go(open(os.path.join(GO, fname)).read())
    src = re.sub(r'"(\\.|[^"\\])*"|`[^`]*`', '""', src)
    hits = [p for p in POST_113 if re.search(p, src)]
    assert not hits, "%s uses APIs newer than go 1.13: %s" % (fname, hits)


# The v1alpha1 plugin interfaces the shim implements (framework/v1alpha1/interface.go:209-367), as
# (parameter types, result types) with the package qualifier the shim imports the framework under.
PLUGIN_API = {
    "Name": ([], "string"),                                                                     # :209
    "PreFilter": (["context.Context", "*framework.CycleState", "*v1.Pod"], "*framework.Status"),  # :242
    "PreFilterExtensions": ([], "framework.PreFilterExtensions"),                               # :249
    "Filter": (["context.Context", "*framework.CycleState", "*v1.Pod", "*framework.NodeInfo"],
               "*framework.Status"),                                                            # :273
    "Score": (["context.Context", "*framework.CycleState", "*v1.Pod", "string"],
              "(int64, *framework.Status)"),                                                    # :320
    "ScoreExtensions": ([], "framework.ScoreExtensions"),                                       # :323
    "Reserve": (["context.Context", "*framework.CycleState", "*v1.Pod", "string"], "*framework.Status"),  # :336
    "Unreserve": (["context.Context", "*framework.CycleState", "*v1.Pod", "string"], ""),         # :367
}


def _method_sigs(recv):
    out = {}
    for f in _go_files():
        src = _strip_go(open(os.path.join(GO, f)).read())
        for m in re.finditer(r"^func\s+\(\s*\w+\s+\*%s\s*\)\s*(\w+)\s*\(([^)]*)\)\s*([^{]*)\{" % recv, src, flags=re.M):
            params = []
            for part in [p.strip() for p in m.group(2).split(",") if p.strip()]:
                toks = part.split()
                params.append(toks[-1])
            # "a, b int" style groups: a bare name takes the next typed parameter's type
            typed = [p if p[0] in "*[" or "." in p or p in ("string", "int64", "int32", "int", "bool") else None
                     for p in params]
            for i in range(len(typed) - 1, -1, -1):
                if typed[i] is None:
                    typed[i] = typed[i + 1]
            out[m.group(1)] = (typed, " ".join(m.group(3).split()))
    return out


@pytest.mark.parametrize("recv,methods", [("GpuEval", list(PLUGIN_API)), ("GpuScore", ["Name", "Score", "ScoreExtensions"])])
def test_plugin_methods_match_the_v1alpha1_interfaces(recv, methods):
    sigs = _method_sigs(recv)
    for name in methods:
        assert name in sigs, "%s lacks %s" % (recv, name)
        assert sigs[name] == (PLUGIN_API[name][0], PLUGIN_API[name][1]), (recv, name, sigs[name])
