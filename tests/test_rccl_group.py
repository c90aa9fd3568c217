"""The runtime's grouped point-to-point calls (zr_rccl.cpp rccl_grouped), which
both collectives use -- the partitioned-setup exchange and the tile-row gather
(zr_runtime.cpp rccl_exchange, zr_device_gather_tile_rows) -- against a fake
RCCL loaded through ZR_RCCL_LIB (CPU only; no device is touched).

A group is closed exactly when it was opened: a failed ncclGroupStart issues no
op and no ncclGroupEnd; a failed op stops the batch and the group is still
closed; the error reported is the first failure's.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zenith_amd", "csrc")

FAKE = r"""
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static int starts, ends, sends, recvs, depth;
static int fail_at(const char* what) {
    const char* f = getenv("FAKE_RCCL_FAIL");
    return f && !strcmp(f, what);
}
int ncclGetUniqueId(void* id) { memset(id, 0, 128); return 0; }
int ncclCommInitRank(void** c, int n, char id[128], int r) { (void)n; (void)id; (void)r; *c = (void*)1; return 0; }
int ncclCommDestroy(void* c) { (void)c; return 0; }
int ncclGroupStart(void) { if (fail_at("start")) return 3; ++starts; ++depth; return 0; }
int ncclGroupEnd(void) { ++ends; if (depth <= 0) return 5; --depth; return fail_at("end") ? 3 : 0; }
int ncclSend(const void* b, size_t n, int t, int p, void* c, void* s) {
    (void)b; (void)n; (void)t; (void)c; (void)s; ++sends; return (fail_at("send") && p == 1) ? 2 : 0; }
int ncclRecv(void* b, size_t n, int t, int p, void* c, void* s) {
    (void)b; (void)n; (void)t; (void)p; (void)c; (void)s; ++recvs; return 0; }
const char* ncclGetErrorString(int r) { return r == 2 ? "send failed" : r == 3 ? "group call failed" : "unbalanced"; }
void fake_counts(int* out) { out[0] = starts; out[1] = ends; out[2] = sends; out[3] = recvs; out[4] = depth; }
"""

DRIVER = r"""
#include <dlfcn.h>
#include <cstdio>
#include <string>
#include "zr_rccl.h"
int main() {
    std::string err;
    if (!zr::rccl_load(err)) { printf("load failed: %s\n", err.c_str()); return 2; }
    char buf[64];
    // ranks 0..3 of an exchange: a send and a receive per peer
    zr::P2POp ops[8];
    for (int p = 0; p < 4; ++p) {
        ops[2 * p] = zr::P2POp{buf, 16, p, true};
        ops[2 * p + 1] = zr::P2POp{buf + 32, 16, p, false};
    }
    const bool ok = zr::rccl_grouped(ops, 8, (void*)1, nullptr, err);
    void* lib = dlopen(getenv("ZR_RCCL_LIB"), RTLD_NOW | RTLD_NOLOAD);
    auto counts = (void (*)(int*))dlsym(lib, "fake_counts");
    int c[5];
    counts(c);
    printf("ok=%d starts=%d ends=%d sends=%d recvs=%d depth=%d err=%s\n", ok ? 1 : 0, c[0], c[1], c[2], c[3], c[4],
           err.c_str());
    return 0;
}
"""


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("rcclgroup")
    (d / "fake.c").write_text(FAKE)
    (d / "driver.cpp").write_text(DRIVER)
    fake = str(d / "libfakercclx.so")
    subprocess.run(["gcc", "-shared", "-fPIC", "-Wall", "-o", fake, str(d / "fake.c")], check=True)
    exe = str(d / "driver")
    subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", "-I", CSRC, "-x", "hip", "--offload-arch=gfx950",
                    str(d / "driver.cpp"), os.path.join(CSRC, "zr_rccl.cpp"), "-ldl", "-o", exe], check=True)
    return exe, fake


def run(driver, fail=None):
    exe, fake = driver
    env = dict(os.environ, ZR_RCCL_LIB=fake)
    env.pop("FAKE_RCCL_FAIL", None)
    if fail:
        env["FAKE_RCCL_FAIL"] = fail
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    fields = dict(kv.split("=", 1) for kv in r.stdout.split(" err=")[0].split())
    return {k: int(v) for k, v in fields.items()}, r.stdout.split(" err=", 1)[1].strip()


def test_group_balanced(driver):
    c, err = run(driver)
    assert c == dict(ok=1, starts=1, ends=1, sends=4, recvs=4, depth=0) and err == ""


def test_failed_start_issues_nothing(driver):
    c, err = run(driver, "start")
    assert c == dict(ok=0, starts=0, ends=0, sends=0, recvs=0, depth=0)
    assert "ncclGroupStart" in err


def test_failed_op_still_closes_the_group(driver):
    c, err = run(driver, "send")
    # ops stop at the failing send (peer 1's), the opened group is closed once
    assert c["ok"] == 0 and c["starts"] == 1 and c["ends"] == 1 and c["depth"] == 0
    assert c["sends"] == 2 and c["recvs"] == 1
    assert "ncclSend" in err and "send failed" in err


def test_failed_end_reported(driver):
    c, err = run(driver, "end")
    assert c["ok"] == 0 and c["starts"] == 1 and c["ends"] == 1
    assert "ncclGroupEnd" in err
