"""Data contracts of the vendored uniception package (reference: /root/reference/uniception) that the MapAnything
path passes between its modules.  Only the dataclasses live here; the modules that consume and produce them are
the MI355X engine's (mapanything/models/mapanything/modules.py), reached as attributes of MapAnything."""
