"""Reference-path shims: with ``galaxy-deconv_amd`` on ``sys.path``,
``from models.Unrolled_ADMM import Unrolled_ADMM`` resolves to the HIP-backed drop-in exactly as
``test.py:12`` imports the reference."""
