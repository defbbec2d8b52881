"""Native (C++) host runtime: the input pipeline (``loader``)."""
