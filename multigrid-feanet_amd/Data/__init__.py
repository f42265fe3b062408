"""Drop-in for the reference's `Data` package (dataset readers, Data/dataset.py)."""
