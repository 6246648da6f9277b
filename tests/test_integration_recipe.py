"""The build recipe of INTEGRATION.md section 1, applied to the reference's
own kv/src/util/CMakeLists.txt.

`integration/kv_util_cmake.patch` is what a maintainer applies: it removes
"crc32c.cc" from UTIL_SRCS -- as the list names it, relative
(kv/src/util/CMakeLists.txt:16) -- BEFORE `add_library(util ...)` (:75) and
links util to libhip_crc32c_batch.so.  The test configures a scratch CMake
project over a copy of the reference's util directory (its sources
symlinked, its CMakeLists.txt copied and patched; nothing is written under
/root/reference and nothing of it is committed) and reads util's SOURCES and
LINK_LIBRARIES back.  It also shows the round-5 snippet (an absolute path,
appended after the library is declared) leaves crc32c.cc in util, so the
reference's static kv::crc32c::Extend would win at link.

CPU only; skipped where the reference tree or cmake is absent (the GPU box).
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_UTIL = "/root/reference/kv/src/util"
PATCH = os.path.join(REPO, "integration", "kv_util_cmake.patch")
LIB = os.path.join(REPO, "wipdb_amd", "lib", "libhip_crc32c_batch.so")

pytestmark = pytest.mark.skipif(
    not os.path.exists(os.path.join(REF_UTIL, "CMakeLists.txt")) or shutil.which("cmake") is None
    or shutil.which("patch") is None,
    reason="needs the reference tree, cmake and patch (this container only)")

TOP = """cmake_minimum_required(VERSION 3.10)
project(hcrc_recipe LANGUAGES C CXX)
set(HCRC_ROOT "{repo}")
add_library(env INTERFACE)
add_subdirectory(kv/src/util)
get_target_property(S util SOURCES)
get_target_property(L util LINK_LIBRARIES)
file(WRITE "${{CMAKE_BINARY_DIR}}/util_sources.txt" "${{S}}")
file(WRITE "${{CMAKE_BINARY_DIR}}/util_links.txt" "${{L}}")
"""


def _tree(tmp, patch=None, append=None, expect_ok=True):
    util = tmp / "kv" / "src" / "util"
    util.mkdir(parents=True)
    for name in os.listdir(REF_UTIL):
        if name != "CMakeLists.txt":
            os.symlink(os.path.join(REF_UTIL, name), util / name)
    shutil.copy(os.path.join(REF_UTIL, "CMakeLists.txt"), util / "CMakeLists.txt")
    if patch:
        subprocess.run(["patch", "-p1", "-d", str(tmp), "-i", patch], check=True,
                       capture_output=True, text=True)
    if append:
        with open(util / "CMakeLists.txt", "a") as f:
            f.write("\n" + append)
    (tmp / "CMakeLists.txt").write_text(TOP.format(repo=REPO))
    build = tmp / "build"
    r = subprocess.run(["cmake", "-S", str(tmp), "-B", str(build)], capture_output=True, text=True)
    if not expect_ok:
        assert r.returncode != 0
        return r.stdout + r.stderr
    assert r.returncode == 0, r.stdout + r.stderr
    srcs = (build / "util_sources.txt").read_text().split(";")
    links = (build / "util_links.txt").read_text().split(";")
    return [os.path.basename(s) for s in srcs], links


def test_reference_util_builds_crc32c(tmp_path):
    srcs, _ = _tree(tmp_path)
    assert "crc32c.cc" in srcs  # the reference as it stands


def test_patch_takes_crc32c_out_of_util_and_links_the_product(tmp_path):
    srcs, links = _tree(tmp_path, patch=PATCH)
    assert "crc32c.cc" not in srcs
    assert "crc32c.h" in srcs and "coding.cc" in srcs  # the rest of util is untouched
    assert LIB in links and "env" in links


def test_round5_snippet_did_not_remove_crc32c(tmp_path):
    """The recipe INTEGRATION.md held until round 5, appended as written: its
    removal (an absolute path, after add_library) leaves crc32c.cc in util,
    and its keyword-form link next to util's plain one does not configure."""
    rm = "list(REMOVE_ITEM UTIL_SRCS ${CMAKE_CURRENT_SOURCE_DIR}/crc32c.cc)\n"
    link = "target_link_libraries(util PUBLIC ${HCRC_ROOT}/wipdb_amd/lib/libhip_crc32c_batch.so)\n"
    srcs, _ = _tree(tmp_path / "a", append=rm)
    assert "crc32c.cc" in srcs
    err = _tree(tmp_path / "b", append=rm + link, expect_ok=False)
    assert "target_link_libraries" in err


def test_patch_text_is_in_integration_md():
    with open(os.path.join(REPO, "INTEGRATION.md")) as f:
        doc = f.read()
    with open(PATCH) as f:
        body = [ln for ln in f.read().splitlines() if ln.startswith(("+", "-"))
                and not ln.startswith(("+++", "---"))]
    for ln in body:
        assert ln in doc, f"INTEGRATION.md does not show the patch line {ln!r}"
