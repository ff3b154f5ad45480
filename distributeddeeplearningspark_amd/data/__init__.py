"""Data plane: synthetic datasets of the reference's and the north-star shapes, and
the pinned-host -> HBM ingest pipeline."""
