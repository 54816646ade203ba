"""The Java drop-in (java/, Panama FFM) against the C-ABI it binds (include/cpg.h).

The image has no JDK, so the Java sources are not compiled or run: this test
checks what can be checked without one.  (1) Every StructLayout declared in Cpg.java has the
C struct's sizeof and every named member the C offsetof — from a probe compiled here with gcc
against include/cpg.h.  (2) Every downcall's FunctionDescriptor has the C prototype's arity and
argument kinds (ADDRESS = a pointer, JAVA_LONG = int64_t, JAVA_INT = int)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "src", "org", "apache", "mahout", "classifier",
                    "sequencelearning", "hmm", "hadoop", "Cpg.java")
HEADER = os.path.join(ROOT, "include", "cpg.h")
SIZES = {"JAVA_DOUBLE": 8, "JAVA_LONG": 8, "JAVA_INT": 4}


def java_layouts():
    src = open(JAVA).read()
    out = {}
    for m in re.finditer(r"StructLayout\s+\w+\s*=\s*MemoryLayout\.structLayout\((.*?)\)\s*"
                         r"\.withName\(\"(\w+)\"\);", src, re.S):
        body, name = m.group(1), m.group(2)
        fields, off = [], 0
        for f in re.finditer(r"sequenceLayout\((\d+),\s*(JAVA_\w+)\)\.withName\(\"(\w+)\"\)|"
                             r"(?<![\w(])(JAVA_\w+)\.withName\(\"(\w+)\"\)", body):
            if f.group(1):
                size, fname = int(f.group(1)) * SIZES[f.group(2)], f.group(3)
            else:
                size, fname = SIZES[f.group(4)], f.group(5)
            fields.append((fname, off))
            off += size
        out[name] = (off, fields)
    return out


def c_layouts(tmp_path, layouts):
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void) {"]
    for s, (_, fields) in layouts.items():
        lines.append(f'  printf("{s} sizeof %zu\\n", sizeof({s}));')
        for f, _ in fields:
            lines.append(f'  printf("{s} {f} %zu\\n", offsetof({s}, {f}));')
    lines += ["  return 0;", "}"]
    c = tmp_path / "probe.c"
    c.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(c)], check=True)
    res = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n"):
        if ln:
            s, f, v = ln.split()
            res[(s, f)] = int(v)
    return res


def test_struct_layouts_match_header(tmp_path):
    jl = java_layouts()
    assert set(jl) == {"cpg_model", "cpg_counts_f64", "cpg_counts_i64", "cpg_island"}
    cl = c_layouts(tmp_path, jl)
    for s, (size, fields) in jl.items():
        assert cl[(s, "sizeof")] == size, s
        for f, off in fields:
            assert cl[(s, f)] == off, (s, f)


def c_prototypes():
    src = re.sub(r"/\*.*?\*/", " ", open(HEADER).read(), flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(int|void|const char\*)\s+(cpg_\w+)\s*\(([^)]*)\)\s*;", src):
        args = [a.strip() for a in m.group(3).split(",") if a.strip() and a.strip() != "void"]
        kinds = []
        for a in args:
            if "*" in a:
                kinds.append("ADDRESS")
            elif re.match(r"(const\s+)?int64_t\b", a):
                kinds.append("JAVA_LONG")
            elif re.match(r"(const\s+)?(int|int32_t)\b", a):
                kinds.append("JAVA_INT")
            else:
                kinds.append("?" + a)
        ret = {"int": "JAVA_INT", "const char*": "ADDRESS", "void": None}[m.group(1)]
        protos[m.group(2)] = (ret, kinds)
    return protos


def test_downcall_descriptors_match_prototypes():
    src = open(JAVA).read()
    protos = c_prototypes()
    calls = re.findall(r"h\(\"(cpg_\w+)\",\s*FunctionDescriptor\.of\(([^;]*?)\)\);", src, re.S)
    assert len(calls) >= 6
    for name, desc in calls:
        kinds = [k.strip() for k in desc.split(",")]
        assert name in protos, name
        ret, args = protos[name]
        assert kinds[0] == ret, (name, kinds[0], ret)
        assert kinds[1:] == args, (name, kinds[1:], args)


@pytest.mark.parametrize("fname", ["GpuHmmEvaluator.java", "GpuBaumWelchMapper.java",
                                   "GpuBaumWelchReducer.java"])
def test_adapters_present(fname):
    src = open(os.path.join(os.path.dirname(JAVA), fname)).read()
    assert "package org.apache.mahout.classifier.sequencelearning.hmm.hadoop;" in src
    assert "NOT COMPILED OR RUN" in src
