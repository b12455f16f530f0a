"""Host logic (CPU): the frame loop's host pool (bundlefusion_amd/csrc/host_pool.h), compiled on its own
with g++: every index of [0, n) visited exactly once per parallel_for, for many consecutive dispatches
of varying sizes (the pool's generation hand-off), from one and from two calling threads, at 1-8 threads (bf_set_host_threads)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "bundlefusion_amd", "csrc")

PROG = r"""
#include "host_pool.h"
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
using namespace bf;
static int run(int seed) {
    std::vector<std::atomic<int>> hit(20000);
    for (int it = 0; it < 3000; it++) {
        const size_t n = (size_t)((it * 7919 + seed * 104729) % 20000);
        for (size_t i = 0; i < n; i++) hit[i].store(0, std::memory_order_relaxed);
        HostPool::get().parallel_for(n, [&](size_t b, size_t e) {
            for (size_t i = b; i < e; i++) hit[i].fetch_add(1, std::memory_order_relaxed);
        }, 64);
        for (size_t i = 0; i < n; i++)
            if (hit[i].load() != 1) { std::printf("bad: it %d n %zu i %zu hit %d\n", it, n, i, hit[i].load()); return 1; }
    }
    return 0;
}
int main(int argc, char** argv) {
    if (argc > 1) HostPool::requested().store(std::atoi(argv[1]));  // bf_set_host_threads
    int r0 = 0, r1 = 0;
    std::thread t([&] { r1 = run(1); });
    r0 = run(0);
    t.join();
    if (r0 || r1) return 1;
    std::printf("ok %d threads\n", HostPool::get().threads());
    return 0;
}
"""


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("pool")
    src, out = d / "pool.cpp", d / "pool"
    src.write_text(PROG)
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", f"-I{CSRC}", str(src), "-o", str(out)], check=True)
    return str(out)


@pytest.mark.parametrize("threads", ["1", "2", "4", "8"])
def test_parallel_for_visits_every_index_once(exe, threads):
    r = subprocess.run([exe, threads], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == f"ok {threads} threads"
