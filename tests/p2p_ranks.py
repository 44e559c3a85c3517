"""Rank processes of the multi-process SQ_COMM_P2P tests (tests/test_gpu_p2p.py).

The ranks are forked by a multiprocessing fork server that conftest.py starts
before the test process touches the GPU, so no process that has initialised
HIP ever forks+execs.  Each rank creates its slab context, sends its handle
blob to the parent, receives every rank's blob, connects, runs the script the
test gave it and sends back what it observed.
"""
import os
import traceback


def rank_main(conn, rank, nranks, shape, kw, env, script):
    lat = None
    try:
        os.environ.update(env)
        from stochquant_amd import Phi4Lattice
        lat = Phi4Lattice(shape, comm="p2p", nranks=nranks, rank=rank, device=0, **kw)
        conn.send(("blob", lat.p2p_handle()))
        blobs = conn.recv()
        lat.p2p_connect(blobs)
        out = {"z0": lat.z0, "nz": lat.nz_local, "ghost": lat.ghost}
        for op, arg in script:
            if op == "upload":
                lat.upload(arg[lat.z0:lat.z0 + lat.nz_local])
            elif op == "upload_r0":   # rank 0 uploads its slab of arg = (field, nranks); the others
                                      # re-upload their own slab (uploads are collective, stochquant.h)
                if rank == 0:
                    lat.upload(arg[0][lat.z0:lat.z0 + lat.nz_local])
                else:
                    lat.upload(lat.download())
            elif op == "step":
                lat.step(arg)
            elif op == "frame":
                out.setdefault("stable", []).append(bool(lat.run_frame()))
                out.setdefault("dtau", []).append(lat.dtau)
                st = lat.stability()
                out.setdefault("fired", []).append(st["fired"])
                out.setdefault("TV", []).append((float(st["T"]), float(st["V"])))
            elif op == "field":
                out.setdefault("field", []).append(lat.download())
            elif op == "correlator":
                out["correlator"] = lat.correlator(arg)
            elif op == "ghost":
                out["ghost"] = lat.ghost
                out["schedule"] = lat.schedule
            else:
                raise ValueError(op)
        out["step_counter"] = lat.step_counter
        out["perf"] = lat.perf()
        lat.close()
        lat = None
        conn.send(("ok", out))
    except Exception:  # reported to the parent, which fails the test
        conn.send(("error", traceback.format_exc()))
    finally:
        if lat is not None:
            lat.close()
        conn.close()


def run_cmd(conn, argv, env, timeout):
    """Run a command from the fork server (a process that never touched the GPU)
    and send back (returncode, stdout, stderr)."""
    import subprocess
    try:
        r = subprocess.run(argv, capture_output=True, text=True, timeout=timeout, env=env)
        conn.send((r.returncode, r.stdout, r.stderr))
    except Exception:
        conn.send((-1, "", traceback.format_exc()))
    finally:
        conn.close()
