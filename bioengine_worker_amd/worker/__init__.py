"""The BioEngine worker service (L6) and code executor."""
