"""Hygiene: the kernel-selection switches the library accepts
(turtle.cpp turtle_set_option), the ones INTEGRATION.md §3 documents and the ones the variant tests
run are the same set - no switch-only kernel without an owning test, no documented switch the
library does not have. CPU only (reads the sources)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(*p):
    with open(os.path.join(ROOT, *p)) as f:
        return f.read()


def _lib_switches():
    src = _read("turtlevsr_amd", "csrc", "turtle.cpp")
    body = src[src.index("int turtle_set_option("):]
    body = body[:body.index("unknown option")]
    return set(re.findall(r'n == "(\w+)"', body))


def _documented():
    doc = _read("INTEGRATION.md")
    sec = doc[doc.index("## 3. Kernel-selection switches"):doc.index("## 4.")]
    return set(re.findall(r"^\| `(\w+)` \|", sec, re.M))


def _tested():
    src = _read("tests", "test_hip_parity.py")
    names = set()
    for fn in ("test_kernel_variants_agree", "test_sab_av_variants_bit_identical", "test_biasfree_layernorm_gemm_variants",
               "test_clip_bf16_psnr_gffn_forced"):
        body = src[src.index(f"def {fn}("):]
        nxt = body.find("\ndef ", 1)
        body = body if nxt < 0 else body[:nxt]
        names |= set(re.findall(r'\b(\w+)=', body)) | set(re.findall(r'"(\w+)":', body))
    return names


def test_switches_documented_and_tested():
    lib, doc, tested = _lib_switches(), _documented(), _tested()
    assert len(lib) >= 30, lib
    assert lib == doc, (sorted(lib - doc), sorted(doc - lib))
    assert lib <= tested, sorted(lib - tested)
