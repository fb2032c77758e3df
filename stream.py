"""Streaming map/reduce driver over tar shards: the MI355X
counterpart of the reference's Hadoop mapper.py / reducer.py.

    python stream.py --list tests/golden/list_tars.txt [--detections]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 stream.py --list list_tars.txt

See tmr_amd/mapreduce.py (template-matching-and-regression-mapreduce_amd/).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tmr_import import load_package  # noqa: E402

load_package()
from tmr_amd.mapreduce import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
