"""Drop-in replacement for ``simple_knn`` (submodules/simple-knn):
``from simple_knn._C import distCUDA2`` (scene/gaussian_model.py:20,134)."""
