"""The drop-in binding compiles against the reference's own headers.

integration/topology_shdnet.c defines the routing API of
routing/topology.h:17-28, integration/worker_send_shdnet.c the
worker_sendPacket of core/worker.h:78 and integration/manager_round_shdnet.c
the round boundary of manager_run; all three call include/shdnet.h.  Compiling
them (gcc -fsyntax-only) against the reference's headers and glib catches a
drift on either side: a changed topology.h / worker.h signature is a
conflicting definition, a changed shdnet.h prototype a wrong call.  The
mutation cases show that the check does catch both kinds.  CPU-only; skipped
where the reference tree or glib's headers are absent (the GPU box).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
GLIB = ["/opt/conda/include/glib-2.0", "/opt/conda/lib/glib-2.0/include"]
FILES = ["topology_shdnet.c", "worker_send_shdnet.c", "manager_round_shdnet.c"]

pytestmark = pytest.mark.skipif(
    not (os.path.isdir(os.path.join(REF, "main/routing")) and all(os.path.isdir(g) for g in GLIB)
         and shutil.which("gcc")),
    reason="reference headers / glib headers / gcc not available")


def compile_c(src_path):
    cmd = ["gcc", "-std=gnu11", "-fsyntax-only", "-Wall", "-Wno-unused-parameter",
           "-Werror=incompatible-pointer-types", "-Werror=int-conversion", "-Werror=implicit-function-declaration",
           "-I", REF, "-I", os.path.join(REF, "main/bindings/c"), "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "integration")] + [f"-I{g}" for g in GLIB] + [src_path]
    return subprocess.run(cmd, capture_output=True, text=True)


@pytest.mark.parametrize("name", FILES)
def test_binding_compiles_against_reference_headers(name):
    r = compile_c(os.path.join(ROOT, "integration", name))
    assert r.returncode == 0, r.stderr
    assert "warning" not in r.stderr, r.stderr


def _mutated(tmp_path, name, pattern, repl):
    src = open(os.path.join(ROOT, "integration", name)).read()
    out, n = re.subn(pattern, repl, src, count=1)
    assert n == 1, pattern
    p = tmp_path / name
    p.write_text(out)
    return compile_c(str(p))


def test_topology_h_signature_drift_is_caught(tmp_path):
    # the wrapper's definition no longer matches topology.h:26
    r = _mutated(tmp_path, "topology_shdnet.c", r"gdouble topology_getLatency\(Topology\* top,",
                 "gdouble topology_getLatency(Topology* top, int extra,")
    assert r.returncode != 0 and "conflicting types" in r.stderr


def test_worker_h_signature_drift_is_caught(tmp_path):
    r = _mutated(tmp_path, "worker_send_shdnet.c", r"void worker_sendPacket\(Host\* srcHost, Packet\* packet\)",
                 "void worker_sendPacket(Host* srcHost, const Packet* packet)")
    assert r.returncode != 0 and "conflicting types" in r.stderr


def test_shdnet_h_call_drift_is_caught(tmp_path):
    # a call that no longer matches include/shdnet.h's prototype
    r = _mutated(tmp_path, "worker_send_shdnet.c", r"shd_round_append_worker\(topology_shdnetHandle\(worker_getTopology\(\)\), w, &rec, 1\)",
                 "shd_round_append_worker(topology_shdnetHandle(worker_getTopology()), &rec, 1)")
    assert r.returncode != 0
