from .dataset import CrowdDataset, SyntheticCrowdDataset  # noqa: F401
from .density import gaussian_filter_density, density_map_gpu  # noqa: F401
from .synthetic import make_synthetic_batch  # noqa: F401
