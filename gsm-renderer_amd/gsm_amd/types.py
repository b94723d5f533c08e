"""numpy views of the reference wire formats (Sources/RendererTypes/include/BridgingTypes.h)."""
import numpy as np

# BridgingTypes.h:57-64 PackedWorldGaussian, 48 B
WORLD32 = np.dtype([("px", "<f4"), ("py", "<f4"), ("pz", "<f4"), ("opacity", "<f4"),
                    ("sx", "<f4"), ("sy", "<f4"), ("sz", "<f4"), ("pad0", "<f4"),
                    ("rot", "<f4", (4,))])
# BridgingTypes.h:66-73 PackedWorldGaussianHalf, 32 B (fp16 fields as raw bits)
WORLD16 = np.dtype([("px", "<f4"), ("py", "<f4"), ("pz", "<f4"), ("opacity", "<u2"),
                    ("sx", "<u2"), ("sy", "<u2"), ("sz", "<u2"), ("rx", "<u2"), ("ry", "<u2"),
                    ("rz", "<u2"), ("rw", "<u2"), ("pad0", "<u2"), ("pad1", "<u2")])
# BridgingTypes.h:75-84 GaussianRenderData, 16 B
RENDER_DATA = np.dtype([("meanX", "<u2"), ("meanY", "<u2"), ("theta", "<u2"), ("sigma1", "<u2"),
                        ("sigma2", "<u2"), ("depth", "<u2"), ("colorR", "u1"), ("colorG", "u1"),
                        ("colorB", "u1"), ("opacity", "u1")])
assert WORLD32.itemsize == 48 and WORLD16.itemsize == 32 and RENDER_DATA.itemsize == 16
