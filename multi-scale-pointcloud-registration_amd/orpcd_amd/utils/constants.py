"""Default hyper-parameters — the values of or_pcd/utils/constants.py:26-81."""
import math

# outlier removal (SOR, constants.py:30-37)
__NB_NEIGHBOURS__ = 64
__STD_RATIO__ = 2
# downsamplers (constants.py:41-56)
__RANDOM_SAMPLE_SIZE__ = 15000
__FARTHEST_SAMPLE_SIZE__ = 10000
__VOXEL_SAMPLE_SIZE__ = 2000
__BASE_VOXEL_SIZE__ = 0.01
__MIN_VOXEL_SIZE__ = 0.0001
__DELTA__ = 0.01
__EPS__ = 0.0005
__SAMPLE_SIZE__ = 4096
# fast global optimizer (constants.py:58-66)
__DIVISION_FACTOR__ = 1.4
__TUPLE_SCALE__ = 0.9
__ITERATION_NUMBER__ = 100
__DECREASE_MU__ = True
__NORMAL_ESTIMATE_RADIUS__ = 0.1
__NORMAL_ESTIMATE_KNN__ = 20
__FPFH_RADIUS__ = 0.1
__FPFH_KNN__ = 20
# generalized ICP (constants.py:68-69)
__MAX_ITERATIONS__ = 100
# optimizer general (constants.py:71-72)
__MAXIMUM_CORRESPONDENCE_DISTANCE__ = 0.5
# aligner (constants.py:75-81)
__MULTISTART_ATTEMPTS__ = 30
__ALIGNER_DEG__ = math.pi / 2
__ALIGNER_MU__ = 0.0
__ALIGNER_STD__ = 0.1
__ALIGNER_MAX_ITER__ = 100
__ALIGNER_DELTA__ = 0.2
__ALIGNER_EPS__ = 0.05
# refiner (constants.py:84-85)
__REFINER_MAX_ITER__ = 200
__REFINER_DISTANCE_THRESHOLD__ = 0.5
# Open3D 0.18 defaults the reference relies on implicitly
__ICP_RELATIVE_FITNESS__ = 1e-6
__ICP_RELATIVE_RMSE__ = 1e-6
__GICP_EPSILON__ = 1e-3
__FGR_MAXIMUM_TUPLE_COUNT__ = 1000
