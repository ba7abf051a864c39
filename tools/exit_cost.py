"""Where a drop-in job process's exit time goes (configs[0] block-features job).

The parent writes the configs[0] N5 input (GPU synth in a child), then for each
variant spawns a job process that runs the block-features job body, then tears
down explicitly with timers (ctg_io cache clear, arena frees, ctg_trim, hipDeviceReset
via os._exit or a normal exit), and reports (body, teardown steps, exit) times."""
import json
import multiprocessing as mp
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def job(conn, inp, variant):
    t0 = time.time()
    from harness import workflow
    from cluster_tools_amd import _lib, rag
    t_imp = time.time()
    out = os.path.join(os.path.dirname(inp), 'out_%s.n5' % variant)
    workflow.graph_workflow(inp, 'seg', out, 'graph', (64, 256, 256), max_jobs=1, mode='threads')
    t_graph = time.time()
    workflow.edge_features_workflow(inp, 'bnd', inp, 'seg', out, 'graph', out, 'features', (64, 256, 256),
                                    max_jobs=1, max_jobs_merge=1, mode='threads')
    t_body = time.time()
    tm = {'import': t_imp - t0, 'graph_wf': t_graph - t_imp, 'features_wf': t_body - t_graph}
    lib = _lib.load()
    if variant in ('explicit', 'explicit_exit0'):
        t = time.time(); lib.ctg_io_cache_clear(); tm['cache_clear'] = time.time() - t
        t = time.time()
        with rag._arena_lock:
            for a in rag._arena_pool:
                a.free()
            rag._arena_pool.clear()
        tm['arena_free'] = time.time() - t
        t = time.time(); lib.ctg_trim(); tm['trim'] = time.time() - t
    conn.send((tm, time.time()))
    conn.close()
    if variant.endswith('exit0'):
        os._exit(0)


def main():
    import bench
    d = tempfile.mkdtemp(prefix='ctg_exit_', dir='/dev/shm' if os.path.isdir('/dev/shm') else None)
    try:
        inp = os.path.join(d, 'in.n5')
        from concurrent.futures import ProcessPoolExecutor
        with ProcessPoolExecutor(1, mp_context=mp.get_context('spawn')) as ex:
            ex.submit(bench._config0_write_inputs, inp, (125, 1250, 1250), (64, 256, 256), 10, 0).result()
        ctx = mp.get_context('spawn')
        for variant in ['default', 'explicit', 'explicit_exit0', 'default_exit0', 'default', 'explicit']:
            r, w = ctx.Pipe(duplex=False)
            p = ctx.Process(target=job, args=(w, inp, variant))
            t_start = time.time()
            p.start()
            w.close()
            tm, t_end = r.recv()
            p.join()
            tm['exit'] = time.time() - t_end
            tm['total'] = time.time() - t_start
            tm['variant'] = variant
            tm['exitcode'] = p.exitcode
            print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in tm.items()}), flush=True)
            shutil.rmtree(os.path.join(d, 'out_%s.n5' % variant), ignore_errors=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == '__main__':
    main()
