"""RadiusScaler (reference: or_pcd/Preprocessor/Scalers/radiusScaler.py:18-30).

Centres the cloud on its mean and divides by its max radius; stores mean and
scale on the instance (read back by Aligner.transfrom, Q6).  This fixes the
unit system in which max_correspondence_distance = 0.5 is expressed."""
import numpy as np

from .BaseScaler import BaseScaler


class RadiusScaler(BaseScaler):
    def process(self, cloud: np.ndarray) -> np.ndarray:
        center = np.mean(cloud, axis=0, keepdims=True)
        # == np.max(scipy.spatial.distance.cdist(center, cloud)) (euclidean):
        # the same per-row sum of squares in the same order, and sqrt is
        # monotone and correctly rounded, so the max is taken before it
        # (one sqrt instead of N; ~1 ms less per 50k-point cloud)
        d = cloud - center
        radius = np.sqrt(np.max(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2]))
        self.mean = center
        self.scale = radius
        return d / radius
