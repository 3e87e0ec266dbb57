"""langstream_amd.cli."""
