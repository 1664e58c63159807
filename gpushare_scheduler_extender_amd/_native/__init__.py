"""In-tree native build outputs (.so); see native/build.py."""
