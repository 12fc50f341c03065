"""Run the reference's main.py UNCHANGED with this repository's `models/` plugins.

Python puts a script's own directory first on sys.path, so `python main.py` would import the
reference's models/ package; this runner executes main.py as __main__ with THIS repo first on
sys.path instead (nothing in the reference is modified):

    cd <dir holding dataset/steam_emb/processed_data_<core>/...>
    python /path/to/this/repo/tools/run_reference_main.py /path/to/GCN_Recommendation/main.py \
        train --model_name LightGCN --debug
"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    main_py = os.path.abspath(sys.argv[1])
    sys.argv = [main_py] + sys.argv[2:]
    sys.path.insert(0, REPO)
    sys.dont_write_bytecode = True
    import models.lightgcn  # noqa: F401  (bind `models` to this repo before main.py runs)
    assert os.path.dirname(os.path.abspath(models.lightgcn.__file__)).startswith(REPO)
    runpy.run_path(main_py, run_name="__main__")


if __name__ == "__main__":
    main()
