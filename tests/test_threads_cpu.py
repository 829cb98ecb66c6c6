"""Thread safety of the drop-in lookup boundary (SURVEY.md §8b "Threading").

The reference is called concurrently from every worker thread
(host/syscall/socket.c:808, host/descriptor/tcp.c:392-393, core/worker.c:
539-551) and guards its cache with a GMutex + 3 GRWLocks (topology.c:26-85).
tests/native/hammer.c drives the product's host C (the lookup, release,
counter and round-staging code of libshdnet) from 8 pthreads and checks that
the final state is the one a serial execution in touch order produces; it is
built against tests/native/stub_dev.c (a host-memory stand-in for the device
layer with a fixed synthetic table -- no GPU here), once plain and once with
-fsanitize=thread, which must report nothing.
"""
import os
import subprocess

import pytest

from shadow_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
BUILD = os.path.join(NATIVE, "_build")
HOST_C = ["topology.c", "routes.c", "round.c", "gml.c", "units.c"]


def _build(tsan: bool) -> str:
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "hammer_tsan" if tsan else "hammer")
    srcs = [os.path.join(NATIVE, "hammer.c"), os.path.join(NATIVE, "stub_dev.c")] + \
           [os.path.join(ROOT, "shadow_amd", "csrc", f) for f in HOST_C]
    flags = ["-O1", "-g", "-std=gnu11", "-ffp-contract=off", "-pthread", "-Wall", "-Wno-unused-parameter",
             "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "shadow_amd", "csrc")]
    if tsan:
        flags += ["-fsanitize=thread"]
    # (built under a private name and renamed into place: pytest-xdist
    # workers build the same binary at once and must not run a half-written one)
    tmp = f"{exe}.{os.getpid()}"
    subprocess.check_call(["gcc"] + flags + srcs + ["-o", tmp, "-lm"])
    os.replace(tmp, exe)
    return exe


@pytest.fixture(scope="module")
def binaries():
    return {"plain": _build(False), "tsan": _build(True)}


CASES = {
    "sparse200_undirected": (synth.sparse_graph_gml(200, 0x5EED0701), 1, 600),
    "sparse150_directed_ns": (synth.sparse_graph_gml(150, 0x5EED0702, ns_variant=True, directed=True), 1, 500),
    "complete30_direct": (synth.complete_graph_gml(30, 0x5EED0703), 0, 90),
}


def _run(exe, path, use_sp, hosts, threads, ops, shards):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1")
    return subprocess.run([exe, str(path), str(use_sp), str(hosts), str(threads), str(ops), str(shards)],
                          capture_output=True, text=True, timeout=300, env=env)


# table: 0 host-mirrored, 1 device-resident (lazy release by device pass,
# here the stub's), 2 two shards of a single-process multi-GPU table
@pytest.mark.parametrize("table", [0, 1, 2], ids=["mirror", "resident", "shards2"])
@pytest.mark.parametrize("kind", ["plain", "tsan"])
@pytest.mark.parametrize("case", list(CASES))
def test_concurrent_lookups_serially_consistent(binaries, case, kind, table, tmp_path):
    gml, use_sp, hosts = CASES[case]
    if table and not use_sp:
        pytest.skip("device-resident tables need use_shortest_path")
    path = tmp_path / "g.gml"
    path.write_text(gml)
    ops = 20000 if kind == "plain" else 4000
    r = _run(binaries[kind], path, use_sp, hosts, 8, ops, table)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert " bad 0 0 0 0" in r.stdout
    if use_sp:
        touched = int(r.stdout.split("touched ")[1].split()[0])
        assert touched > 10  # many rows were released concurrently


@pytest.mark.parametrize("case", ["sparse200_undirected", "sparse150_directed_ns"])
def test_single_worker_release_sequence_same_for_every_table(binaries, case, tmp_path):
    """One worker (the reference's serial order): the device-resident and the
    two-shard tables release exactly what the host-mirrored table releases --
    same touch order, same min-jump callback sequence (value by value)."""
    gml, use_sp, hosts = CASES[case]
    path = tmp_path / "g.gml"
    path.write_text(gml)
    outs = []
    for table in (0, 1, 2):
        r = _run(binaries["plain"], path, use_sp, hosts, 1, 20000, table)
        assert r.returncode == 0, r.stdout + r.stderr[-3000:]
        outs.append(r.stdout.split("cb_calls ")[1].split(" staged")[0] + r.stdout.split("touched ")[1].split()[0])
    assert outs[0] == outs[1] == outs[2], outs
