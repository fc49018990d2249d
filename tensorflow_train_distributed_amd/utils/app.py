"""`tf.app.run()` equivalent (/root/reference/distribute_training.py:241-242): parse the
command line into FLAGS, then call main(argv) with the unparsed remainder and exit with its
return code."""
from __future__ import annotations

import sys

from .flags import FLAGS


def run(main=None, argv=None):
    argv = list(sys.argv if argv is None else argv)
    rest = FLAGS(argv)
    if main is None:
        main = sys.modules["__main__"].main
    rc = main(rest)
    return rc


def run_and_exit(main=None, argv=None):
    sys.exit(run(main, argv))
