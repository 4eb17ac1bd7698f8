{{- define "chat-ai.name" -}}{{ .Release.Name }}{{- end -}}
{{- define "chat-ai.pullSecret" -}}{{ default (printf "%s-registry" .Chart.Name) .Values.imagePullSecret }}{{- end -}}
{{- define "chat-ai.splitMode" -}}{{ if gt (int .Values.gpu.perPod) 1 }}row{{ else }}{{ .Values.engine.splitMode }}{{ end }}{{- end -}}
