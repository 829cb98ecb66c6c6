"""Multi-process rank harness for the world>1 tests: one
spawned process per rank, a torch.distributed gloo group rendezvoused through
a FileStore in the test's tmp_path (no port is chosen, closed and re-bound, so
no other socket on the box can take it), an explicit init timeout, one overall
deadline for the parent, and a `finally` that kills and joins every child
still alive -- so a rank that dies or hangs fails the test within seconds of
the event and leaves nothing behind.

    results = run_ranks(worker, world, tmp_path, args=(...), deadline=120)

`worker(rank, world, *args)` runs inside an initialised default group and
returns a picklable value; results[rank] is that value.  A rank that raises
reports its traceback, which the parent re-raises at once (its peers are
killed, not waited for)."""
import datetime
import os
import queue
import time
import traceback

INIT_TIMEOUT_S = 60


class RankFailed(AssertionError):
    pass


def _entry(target, rank, world, init_method, q, args, env):
    os.environ.update(env)
    if os.environ.get("SHD_TEST_DIE_RANK") == str(rank):  # the harness's own failure test
        os._exit(3)
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", init_method=init_method, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=INIT_TIMEOUT_S))
        val = target(rank, world, *args)
        q.put((rank, val, None))
    except BaseException:
        q.put((rank, None, traceback.format_exc()))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_ranks(target, world, tmp_path, args=(), env=None, deadline=120.0, poll=0.5):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = "file://" + os.path.join(str(tmp_path), "rdzv_%d" % time.monotonic_ns())
    procs = [ctx.Process(target=_entry, args=(target, r, world, init, q, tuple(args), dict(env or {})), daemon=True)
             for r in range(world)]
    results = {}
    t_end = time.monotonic() + deadline
    try:
        for p in procs:
            p.start()
        while len(results) < world:
            try:
                rank, val, err = q.get(timeout=poll)
            except queue.Empty:
                dead = [(r, p.exitcode) for r, p in enumerate(procs)
                        if p.exitcode is not None and r not in results]
                if dead:
                    # a late put from a rank that just exited may still be in the pipe
                    try:
                        rank, val, err = q.get(timeout=2 * poll)
                    except queue.Empty:
                        raise RankFailed("rank %d exited with code %s before reporting" % dead[0]) from None
                elif time.monotonic() > t_end:
                    raise RankFailed("ranks %s did not report within %.0f s"
                                     % (sorted(set(range(world)) - set(results)), deadline))
                else:
                    continue
            if err:
                raise RankFailed("rank %d failed:\n%s" % (rank, err))
            results[rank] = val
        for p in procs:
            p.join(timeout=max(1.0, t_end - time.monotonic()))
        bad = [(r, p.exitcode) for r, p in enumerate(procs) if p.exitcode != 0]
        if bad:
            raise RankFailed("rank %d exit code %s after reporting" % bad[0])
        return [results[r] for r in range(world)]
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
        for p in procs:
            if p.pid is not None:
                p.join(timeout=10)
        q.cancel_join_thread()
        q.close()
