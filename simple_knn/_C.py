"""``simple_knn._C.distCUDA2`` (knn/ext.cpp, knn/spatial.cu:14-24) on MI355X."""
from gaussian_splatting_with_eye_tracking_amd._C import distCUDA2  # noqa: F401
