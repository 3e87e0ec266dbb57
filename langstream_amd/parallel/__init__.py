"""langstream_amd.parallel."""
