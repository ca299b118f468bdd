"""Drop-in for the reference package `wrinklefree_inference` -- the hot-path subpackages only:
`kernels` (src/wrinklefree_inference/kernels) and `kv_cache` (src/wrinklefree_inference/kv_cache),
backed by the gfx950 HIP kernels of lib/libwfbitnet.so. Client/server/cache/MoE subsystems of the
reference are out of scope."""
__version__ = "0.1.0+mi355x"
