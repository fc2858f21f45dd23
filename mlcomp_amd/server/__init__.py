"""Server side: scheduler (supervisor) and REST API."""
