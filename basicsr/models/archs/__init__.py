"""Arch plug-ins resolved by ``import_module('basicsr.models.archs.' + opt['model'].lower())``
(video_restoration_model.py:18-21): turtle_t1_arch, turtlesuper_t1_arch."""
