"""MI355X-native drop-in for the ``simple_knn`` package (``from simple_knn._C import distCUDA2``,
reference geometry/gaussian_base.py:25 and five other geometry modules)."""
