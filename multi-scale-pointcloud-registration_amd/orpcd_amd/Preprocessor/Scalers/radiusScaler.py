"""RadiusScaler (reference: or_pcd/Preprocessor/Scalers/radiusScaler.py:18-30).

Centres the cloud on its mean and divides by its max radius; stores mean and
scale on the instance (read back by Aligner.transfrom, Q6).  This fixes the
unit system in which max_correspondence_distance = 0.5 is expressed."""
import numpy as np

from .BaseScaler import BaseScaler


class RadiusScaler(BaseScaler):
    def process(self, cloud: np.ndarray) -> np.ndarray:
        center = np.mean(cloud, axis=0, keepdims=True)
        # == np.max(scipy.spatial.distance.cdist(center, cloud)) (euclidean)
        radius = np.max(np.sqrt(((cloud - center) ** 2).sum(axis=1)))
        self.mean = center
        self.scale = radius
        return (cloud - center) / radius
