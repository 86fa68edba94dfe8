"""Control arm of the cross-stream ingest check (r03ag): the device ingest with
its copy-stream -> parse-stream ordering (ingest_device.XSTREAM_WAIT) switched
off, on the batch-alternating split of tests/test_gpu_ingest.py.  Run once; the
product path keeps the wait on."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from grid_amd.utils import ingest_device

ingest_device.XSTREAM_WAIT = False
sys.exit(pytest.main(["-x", "-q", "-p", "no:cacheprovider", "tests/test_gpu_ingest.py", "-k", "batches or model"]))
