"""VideoPrism video encoder on AMD MI355X (gfx950).

Drop-in for the reference package `videoprism` (tmoroney/videoprism-mlx): the modules
`models`, `models_mlx`, `utils` keep the reference's names and signatures; the forward
pass runs in hand-written HIP kernels (libvideoprism_hip.so, C-ABI in
include/videoprism_hip.h) loaded through `videoprism._native`.
"""

__version__ = "0.1.0"
