"""Recipe (test infrastructure): build the reference's Cython rating-SGD module
/root/reference/util/matrix_factorization.pyx (SVD, RSVD, SVDpp) into oracle/_ref/.

The source is compiled where it lies (read-only): cythonize writes its generated C under
oracle/_ref/build and the extension into oracle/_ref/ (git-ignored).  Used only to generate the
golden fixtures of tests/golden/make_golden_mf.py in the build container; the GPU box never has
/root/reference and never runs this.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/util/matrix_factorization.pyx"
OUT = os.path.join(HERE, "_ref")


def build():
    import numpy as np
    from Cython.Build import cythonize
    from setuptools import Extension
    from setuptools.dist import Distribution

    os.makedirs(OUT, exist_ok=True)
    ext = Extension("matrix_factorization", [SRC], include_dirs=[np.get_include()])
    mods = cythonize([ext], build_dir=os.path.join(OUT, "build"), quiet=True,
                     compiler_directives={"language_level": 3})
    dist = Distribution({"ext_modules": mods})
    cmd = dist.get_command_obj("build_ext")
    cmd.build_lib = OUT
    cmd.build_temp = os.path.join(OUT, "build", "tmp")
    cmd.ensure_finalized()
    cmd.run()
    return OUT


if __name__ == "__main__":
    print(build(), file=sys.stderr)
