"""PyTorch adapter of the engine (reference: src/py/ddl/tensorflow/)."""
