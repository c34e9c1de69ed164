"""Network helpers (reference utils/network.py)."""

import socket

from .utils import log


def is_udp_port_available(port):
  try:
    sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sock.bind(('', port))
    sock.close()
  except OSError as exc:
    log.warning('UDP port %d cannot be used %s', port, exc)
    return False
  return True


def find_available_udp_port(start=40300, count=1000):
  for p in range(start, start + count):
    if is_udp_port_available(p):
      return p
  raise RuntimeError('no free UDP port in [%d, %d)' % (start, start + count))
