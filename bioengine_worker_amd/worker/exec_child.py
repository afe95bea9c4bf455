"""Child process for ``run_code``: ``python -m bioengine_worker_amd.worker.exec_child IN OUT``."""
import asyncio
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
        (kind, body, fname), args, kwargs = pickle.load(f)
    try:
        if kind == "source":
            from .code_executor import load_func_from_source

            fn = load_func_from_source(body, fname)
        else:
            import cloudpickle

            fn = cloudpickle.loads(body)
            if not callable(fn):
                raise ValueError("the unpickled object is not callable")
        res = fn(*args, **kwargs)
        if asyncio.iscoroutine(res):
            res = asyncio.run(res)
        payload = (True, res, "")
    except BaseException as e:  # noqa: BLE001
        payload = (False, f"{type(e).__name__}: {e}", traceback.format_exc())
        traceback.print_exc()
    import cloudpickle

    try:
        data = cloudpickle.dumps(payload)
    except Exception as e:  # noqa: BLE001
        data = cloudpickle.dumps((False, f"result is not serializable: {e}", ""))
    with open(out + ".tmp", "wb") as f:
        f.write(data)
    os.replace(out + ".tmp", out)


if __name__ == "__main__":
    main()
