"""simple_knn -- MI355X-native `distCUDA2` (used once by GaussianModel.create_from_pcd,
/root/reference/scene/gaussian_model.py:20,134-135)."""
