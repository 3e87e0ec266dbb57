"""langstream_amd.webservice."""
