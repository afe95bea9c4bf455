import sys

from bioengine_worker_amd.worker.__main__ import main

if __name__ == "__main__":
    sys.exit(main())
