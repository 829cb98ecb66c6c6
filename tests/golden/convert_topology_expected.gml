graph [
  directed 1
  node [
    id 0
    label "poi-1"
    country_code "US"
    bandwidth_down "81920 Kibit"
    bandwidth_up "81920 Kibit"
  ]
  edge [
    source 0
    target 0
    latency "50 ms"
    packet_loss 0.0
  ]
]
