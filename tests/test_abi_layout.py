"""The C-ABI structs as a binding sees them: the ctypes mirrors in siddhi_amd/__init__.py must have the size and
field offsets a C compiler gives include/siddhi_amd.h, so the layouts cannot drift apart again (a binding that
allocates a short sdg_out gets an out-of-bounds write from sdg_poll). A tiny C program compiled against the header
prints offsetof / sizeof for every field; the same program pins the Panama layout documented in INTEGRATION.md."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

import siddhi_amd as sa

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "siddhi_amd.h")


def header_fields(struct):
    """field names of `typedef struct <struct> { ... } <struct>;` in declaration order"""
    text = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (struct, struct), text, re.S).group(1)
    names = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        for part in decl.split(","):
            names.append(re.findall(r"([A-Za-z_][A-Za-z0-9_]*)\s*$", part.strip())[0])
    return names


def c_layout(struct, fields):
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"siddhi_amd.h\"\nint main(void) {\n"
    src += '    printf("sizeof %%zu\\n", sizeof(%s));\n' % struct
    for f in fields:
        src += '    printf("%s %%zu\\n", offsetof(%s, %s));\n' % (f, struct, f)
    src += "    return 0;\n}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        exe = os.path.join(d, "t")
        open(c, "w").write(src)
        subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), c, "-o", exe])
        out = subprocess.check_output([exe]).decode().split("\n")
    return dict((ln.split()[0], int(ln.split()[1])) for ln in out if ln.strip())


@pytest.mark.parametrize("struct,mirror", [("sdg_opts", sa._Opts), ("sdg_out", sa._Out), ("sdg_stats", sa.Stats)])
def test_ctypes_mirror_matches_the_header(struct, mirror):
    fields = header_fields(struct)
    lay = c_layout(struct, fields)
    assert [f[0] for f in mirror._fields_] == fields, "field order / names differ from %s" % struct
    assert ctypes.sizeof(mirror) == lay["sizeof"], struct
    for f in fields:
        assert getattr(mirror, f).offset == lay[f], "%s.%s" % (struct, f)


def test_integration_panama_sdg_out_matches_the_header():
    """INTEGRATION.md's Panama StructLayout for sdg_out: every header field, at the C offsets"""
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"StructLayout SDG_OUT = MemoryLayout\.structLayout\((.*?)\);", doc, re.S)
    assert m, "INTEGRATION.md has no SDG_OUT layout"
    size = {"JAVA_LONG": 8, "ADDRESS": 8, "JAVA_INT": 4}
    off, got = 0, {}
    for item in re.findall(r"(JAVA_LONG|ADDRESS|JAVA_INT)\.withName\(\"(\w+)\"\)|paddingLayout\((\d+)\)",
                           m.group(1)):
        kind, name, pad = item
        if pad:
            off += int(pad)
            continue
        got[name] = off
        off += size[kind]
    fields = header_fields("sdg_out")
    lay = c_layout("sdg_out", fields)
    assert set(got) == set(fields)
    for f in fields:
        assert got[f] == lay[f], "SDG_OUT.%s at %d, C offset %d" % (f, got[f], lay[f])
    assert off == lay["sizeof"]
