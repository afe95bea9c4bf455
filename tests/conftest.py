import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels); skipped in CPU CI")
    config.addinivalue_line("markers", "unit: hermetic CPU unit test")
    config.addinivalue_line("markers", "integration: multi-component test against in-process fakes")
    config.addinivalue_line("markers", "end_to_end: full worker/app flow against LocalHypha")
    config.addinivalue_line("markers", "requires_gpu: alias used by reference app tests")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _isolate_app_installs():
    """Apps deployed in-process append their pip ``--target`` directory to ``sys.path``
    (``apps/requirements.py``); undo that after each test so one test's wheelhouse installs (e.g.
    ``bioengine_testdep``) are not importable in the next one."""
    before = list(sys.path)
    mods = set(sys.modules)
    yield
    from bioengine_worker_amd.apps import requirements as _req

    for p in [p for p in sys.path if p not in before]:
        sys.path.remove(p)
        _req._APP_PATHS.discard(p)
    for m in [m for m in sys.modules if m not in mods and m.startswith("bioengine_testdep")]:
        del sys.modules[m]


@pytest.fixture(scope="session")
def gpu():
    import torch

    from bioengine_worker_amd.ops import _native

    assert torch.cuda.is_available()
    _native.hip()  # must load: GPU tests never run on a silent fallback
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def wheelhouse(tmp_path_factory):
    """A local wheelhouse holding ``bioengine-testdep==0.1.0`` (module ``bioengine_testdep``,
    ``VALUE = "wheel-ok"``), built offline with ``pip wheel --no-index``."""
    import subprocess
    import textwrap

    src = tmp_path_factory.mktemp("pkgsrc")
    (src / "bioengine_testdep.py").write_text('VALUE = "wheel-ok"\n')
    (src / "setup.py").write_text(textwrap.dedent("""
        from setuptools import setup
        setup(name="bioengine-testdep", version="0.1.0", py_modules=["bioengine_testdep"])
    """))
    wh = tmp_path_factory.mktemp("wheelhouse")
    subprocess.run([sys.executable, "-m", "pip", "wheel", "--no-index", "--no-deps", "--no-build-isolation",
                    "--disable-pip-version-check", "-w", str(wh), str(src)], check=True, capture_output=True, timeout=300)
    assert list(wh.glob("bioengine_testdep-0.1.0-*.whl"))
    return wh
