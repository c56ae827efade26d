"""The JNI binding sources (java/…/OmrNative.java, jni/omr_jni.c) stay in step
with each other and with include/omr/omr.h.  There is no JDK in this image, so this checks the
sources as text: every `native` method has its JNIEXPORT, and every omr_* function the shim
calls is declared in the header and exported by libomr.so."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(REPO, "java/src/main/java/com/glencoesoftware/omero/ms/image/region/gpu/OmrNative.java")
JNI_C = os.path.join(REPO, "jni/omr_jni.c")
HDR = os.path.join(REPO, "include/omr/omr.h")
PREFIX = "Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_"


def _read(p):
    with open(p) as f:
        return f.read()


def test_every_native_method_has_its_jni_export():
    natives = set(re.findall(r"\bnative\s+[\w\[\]]+\s+(\w+)\s*\(", _read(JAVA)))
    exports = set(re.findall(PREFIX + r"(\w+)\s*\(", _read(JNI_C)))
    assert natives, "no native methods found"
    assert natives == exports, (natives - exports, exports - natives)


def test_shim_calls_only_declared_and_exported_symbols():
    from omr import _lib
    declared = set(re.findall(r"\b(omr_\w+)\s*\(", _read(HDR)))
    src = re.sub(r"/\*.*?\*/", "", _read(JNI_C), flags=re.S)
    hdr = _read(HDR)
    types = set(re.findall(r"}\s*(omr_\w+)\s*;", hdr)) | set(re.findall(r"typedef\s+[\w ]+?\b(omr_\w+)\s*;", hdr))
    called = set(re.findall(r"\b(omr_\w+)\s*\(", src)) - types      # (omr_status)(...) is a cast
    assert called, "the shim calls no omr_* function"
    assert called <= declared, called - declared
    for name in called:
        assert hasattr(_lib.lib, name), name


def test_java_constants_match_header():
    """Every `NAME = value` constant of OmrNative / OmrException whose OMR_NAME exists in omr.h
    (status codes, pixel types, models, families, projections, semantics bits) has its value."""
    hdr = {n: int(v, 0) for n, v in re.findall(r"\b(OMR_[A-Z0-9_]+)\s*=\s*(0x[0-9A-Fa-f]+|\d+)", _read(HDR))}
    for n, sh in re.findall(r"\b(OMR_[A-Z0-9_]+)\s*=\s*1u\s*<<\s*(\d+)", _read(HDR)):
        hdr[n] = 1 << int(sh)
    checked = 0
    for f in ("OmrNative.java", "OmrException.java"):
        java = _read(os.path.join(os.path.dirname(JAVA), f))
        for decl in re.findall(r"static final int ([^;]+);", java):
            for name, val in re.findall(r"\b([A-Z][A-Z0-9_]*)\s*=\s*(0x[0-9A-Fa-f]+|\d+)", decl):
                if "OMR_" + name in hdr:
                    assert int(val, 0) == hdr["OMR_" + name], (f, name, val)
                    checked += 1
    assert checked >= 15, checked


def _canon(name):
    n = name.lower().replace("_", "")
    for key, canon in (("active", "active"), ("family", "family"), ("coefficient", "coefficient"),
                       ("noise", "noise_reduction"), ("reverse", "reverse"), ("windowstart", "start"),
                       ("inputstart", "start"), ("windowend", "end"), ("inputend", "end"), ("globalmin", "gmin"),
                       ("globalmax", "gmax"), ("rgba", "rgba")):
        if key in n:
            return canon
    raise AssertionError(name)


def test_pack_channel_layout_in_lockstep():
    """The 13-double channel record has three writers/readers that must agree field by field:
    OmrNative.packChannel (Java), the shim's load_settings (C) and the mock's pack_channels (the
    test double the GPU shim tests use, tests/jni_mock.py)."""
    java = _read(JAVA)
    body = java[java.index("public static void packChannel"):]
    body = body[:body.index("\n    }\n")]
    jmap = {}
    for idx, expr in re.findall(r"settings\[o(?: \+ (\d+))?(?: \+ k)?\]\s*=\s*(\w+)", body):
        jmap[int(idx or 0)] = _canon(expr)
    assert "settings[o + 9 + k] = rgba[k]" in body
    jmap.update({9 + k: "rgba" for k in range(4)})
    c = _read(JNI_C)
    load = c[c.index("static int load_settings"):]
    load = load[:load.index("\n}\n")]
    cmap = {int(i): _canon(f) for f, i in re.findall(r"b->(\w+)\s*=\s*(?:\(\w+\))?p\[(\d+)\]", load)}
    assert "b->rgba[k] = (uint8_t)(int)p[9 + k]" in load
    cmap.update({9 + k: "rgba" for k in range(4)})
    mock = _read(os.path.join(REPO, "tests", "jni_mock.py"))
    pk = mock[mock.index("def pack_channels"):]
    pk = pk[:pk.index("\n\n\n")]
    lst = pk[pk.index("s[o:o + 13] = ["):pk.index("]\n", pk.index("s[o:o + 13] = ["))]
    items = re.findall(r'"(\w+)"', lst)
    pmap = {i: _canon(n) for i, n in enumerate(items)}
    assert "*d.get(\"rgba\"" in lst
    pmap.update({9 + k: "rgba" for k in range(4)})
    assert len(jmap) == len(cmap) == len(pmap) == 13, (jmap, cmap, pmap)
    assert jmap == cmap == pmap, (jmap, cmap, pmap)
