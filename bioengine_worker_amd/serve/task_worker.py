"""Child process of an isolated remote task: ``python -m bioengine_worker_amd.serve.task_worker IN OUT``."""
import os
import pickle
import sys
import traceback


def main():
    inp, out = sys.argv[1], sys.argv[2]
    sys.path.insert(0, os.getcwd())
    from ..compat import install

    install()
    with open(inp, "rb") as f:
        fn, args, kwargs = pickle.load(f)
    try:
        res = fn(*args, **kwargs)
        payload = (True, res, "")
    except BaseException as e:  # noqa: BLE001
        tb = traceback.format_exc()
        try:
            pickle.dumps(e)
        except Exception:
            e = RuntimeError(f"{type(e).__name__}: {e}")
        payload = (False, e, tb)
    import cloudpickle

    with open(out + ".tmp", "wb") as f:
        f.write(cloudpickle.dumps(payload))
    os.replace(out + ".tmp", out)


if __name__ == "__main__":
    main()
