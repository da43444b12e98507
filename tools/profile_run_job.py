#!/usr/bin/env python3
"""cProfile of IllumstatsCalculator.run_job (GPU decode) on a warm calculator:
where a job's fixed cost goes.  Prints the top functions by cumulative time.
    python tools/profile_run_job.py [--sites 128]"""
import argparse
import cProfile
import os
import pstats
import shutil
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=128)
    ap.add_argument("--decode", default="gpu")
    a = ap.parse_args()
    from tmlibrary_amd.models import file as h5
    from tmlibrary_amd.models.file import ExperimentStore
    from tmlibrary_amd.synth import synth_sites_host
    from tmlibrary_amd.workflow.corilla.api import IllumstatsCalculator
    root = tempfile.mkdtemp(prefix="tmh_prof_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        d = os.path.join(root, "channel_image_files")
        os.makedirs(d)
        sites = synth_sites_host(8, 2160, 2560, seed=99)
        for i in range(a.sites):
            h5.write_channel_image(os.path.join(d, "channel_image_file_%d.h5" % i), sites[i % 8], 4)
        store = ExperimentStore(root)
        batch = {"id": 1, "channel_id": 1, "channel_image_files_ids": [[i] for i in range(a.sites)]}
        calc = IllumstatsCalculator(1, store=store, decode=a.decode)
        calc.run_job(batch)
        calc.run_job(batch)
        pr = cProfile.Profile()
        pr.enable()
        calc.run_job(batch)
        pr.disable()
        print(calc.last_timing)
        pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
